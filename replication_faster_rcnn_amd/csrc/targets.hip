// Target assignment (utils/utils.py:102-276) on gfx950: fp64 IoU matching,
// anchor/proposal labels and numpy-RNG-exact sampling.
//
// IoU: numpy's dtype promotion and op order of utils/utils.py:114-119, in fp64
// (anchors fp32, gt fp64 -> fp64; both fp32 -> fp32).  argmax = first maximum,
// NaN first (numpy rules).
//
// Sampling: the reference calls np.random.choice(arr, k, replace=False) on the
// GLOBAL legacy RandomState (utils/utils.py:194,201,251,258), which is
// arr[permutation(len(arr))[:k]]; permutation is Fisher-Yates
//   for i = n-1 .. 1: j = random_interval(i); swap(a[i], a[j])
// with random_interval = "next MT19937 word & mask(i), reject while > i".
// The caller hands the MT19937 state (624 words + pos) in and gets it back,
// so the numpy global stream continues exactly as after the reference's calls.
//  * one 1024-thread workgroup runs the rejection automaton over 1024-word
//    windows of the stream: thread t owns word t; which words are accepted
//    depends on how many earlier words were, solved as a fixed point over the
//    16 wave prefix counts (a few rounds); state blocks are twisted into an LDS
//    ring ahead of the window (fy_walk / mt_twist);
//  * only the permutation positions the caller needs are reconstructed from
//    the recorded swaps (fy_final): the last m positions for AnchorTarget
//    (which m elements survive the disable), the first k for ProposalTarget
//    (in order).
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "common.h"

namespace frcnn {

// ------------------------------------------------------------------ IoU core
// numpy: tl = max(a[:2], b[:2]); br = min(a[2:], b[2:]);
//        inter = prod(br - tl) * all(tl < br); area_a = prod(a[2:] - a[:2]) (a's dtype)
//        iou = inter / (area_a + area_b - inter)
// np.maximum / np.minimum: NaN propagates.
template <class T>
__device__ __forceinline__ T np_max(T a, T b) { return (a != a || a >= b) ? a : b; }
template <class T>
__device__ __forceinline__ T np_min(T a, T b) { return (a != a || a <= b) ? a : b; }

template <class TA>
__device__ __forceinline__ double iou_np(const TA* a, double area_a_as_f64, const double* b,
                                         double area_b) {
    double tl0 = np_max(static_cast<double>(a[0]), b[0]);
    double tl1 = np_max(static_cast<double>(a[1]), b[1]);
    double br0 = np_min(static_cast<double>(a[2]), b[2]);
    double br1 = np_min(static_cast<double>(a[3]), b[3]);
    double inter = (br0 - tl0) * (br1 - tl1);
    inter = inter * ((tl0 < br0 && tl1 < br1) ? 1.0 : 0.0);
    double uni = area_a_as_f64 + area_b;
    uni = uni - inter;
    return inter / uni;
}

template <class T>
__device__ __forceinline__ T area_np(const T* a) {
    T d0 = a[2] - a[0];
    T d1 = a[3] - a[1];
    return d0 * d1;
}

// numpy max/argmax "better" relation: NaN wins (first NaN), else larger, ties -> earlier.
__device__ __forceinline__ bool np_better(double v, double cur, bool cur_nan) {
    if (cur_nan) return false;
    if (v != v) return true;
    return v > cur;
}

// ------------------------------------------------------------ gt compaction
// Rows with label == -1 are padding (utils/data_loader.py:88-89, train.py:74-76).
__global__ __launch_bounds__(64) void gt_compact_kernel(const double* __restrict__ boxes,
                                                        const double* __restrict__ labels,
                                                        int Gp, double* __restrict__ gt,
                                                        double* __restrict__ gl,
                                                        int* __restrict__ gcount) {
    const int n = blockIdx.x, lane = threadIdx.x;
    int base = 0;
    for (int g0 = 0; g0 < Gp; g0 += 64) {
        const int g = g0 + lane;
        const bool v = g < Gp && labels[static_cast<size_t>(n) * Gp + g] != -1.0;
        const uint64_t bal = __ballot(v);
        if (v) {
            const int o = base + __popcll(bal & lanemask_lt());
            for (int c = 0; c < 4; ++c)
                gt[(static_cast<size_t>(n) * Gp + o) * 4 + c] = boxes[(static_cast<size_t>(n) * Gp + g) * 4 + c];
            gl[static_cast<size_t>(n) * Gp + o] = labels[static_cast<size_t>(n) * Gp + g];
        }
        base += __popcll(bal);
    }
    if (lane == 0) gcount[n] = base;
}

// --------------------------------------------------------- AnchorTarget IoU
constexpr int kMaxG = 256;

struct ArgMax {
    double v;
    int i;
    int nan;
};

__device__ __forceinline__ ArgMax am_combine(ArgMax a, ArgMax b) {  // a precedes b
    if (a.nan) return a;
    if (b.nan) return b;
    if (b.v > a.v) return b;
    return a;
}

// grid (ceil(A/256), N): per anchor row max/argmax over the image's gt, and per
// block the column (max, first anchor) partial of every gt.
__global__ __launch_bounds__(256) void at_iou_kernel(const float* __restrict__ anchors, int A,
                                                     const double* __restrict__ gt,
                                                     const int* __restrict__ gcount, int Gp,
                                                     int32_t* __restrict__ row_arg,
                                                     double* __restrict__ row_max,
                                                     double* __restrict__ col_v,
                                                     int* __restrict__ col_i) {
    __shared__ double sg[kMaxG][4];
    __shared__ double sa[kMaxG];
    __shared__ ArgMax wred[4][kMaxG];
    const int n = blockIdx.y;
    const int G = gcount[n];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int g = tid; g < G; g += 256) {
        for (int c = 0; c < 4; ++c) sg[g][c] = gt[(static_cast<size_t>(n) * Gp + g) * 4 + c];
        sa[g] = area_np(sg[g]);
    }
    __syncthreads();
    const int a = blockIdx.x * 256 + tid;
    const bool va = a < A;
    float box[4] = {0.f, 0.f, 0.f, 0.f};
    if (va)
        for (int c = 0; c < 4; ++c) box[c] = anchors[static_cast<size_t>(a) * 4 + c];
    const double aa = static_cast<double>(area_np(box));  // fp32 product, then promoted
    ArgMax best{0.0, 0, 0};
    for (int g = 0; g < G; ++g) {
        const double v = iou_np(box, aa, sg[g], sa[g]);
        if (g == 0) {
            best.v = v;
            best.i = 0;
            best.nan = v != v;
        } else if (np_better(v, best.v, best.nan)) {
            best.v = v;
            best.i = g;
            best.nan = v != v;
        }
        // column partial: the wave's first anchor with the best value, as the ordered
        // am_combine fold gives it -- the first NaN if any, else the first lane at the
        // maximum (ties and -0.0 / 0.0 keep the earlier lane; the invalid lanes, a
        // suffix, hold -inf and index 0x7fffffff) -- from two ballots and a max
        const double cvv = va ? v : -INFINITY;
        const uint64_t nanb = __builtin_amdgcn_ballot_w64(va && v != v);
        ArgMax c;
        if (nanb) {
            const int f = __ffsll(static_cast<unsigned long long>(nanb)) - 1;
            c = ArgMax{__builtin_nan(""), static_cast<int>(blockIdx.x) * 256 + wid * 64 + f, 1};
        } else {
            double m = cvv;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) m = fmax(m, __shfl_xor(m, o, 64));
            const uint64_t eq = __builtin_amdgcn_ballot_w64(cvv == m);
            const int f = __ffsll(static_cast<unsigned long long>(eq)) - 1;
            const int af = static_cast<int>(blockIdx.x) * 256 + wid * 64 + f;
            c = ArgMax{m, af < A ? af : 0x7fffffff, 0};
        }
        if (lane == 0) wred[wid][g] = c;
    }
    if (va) {
        row_arg[static_cast<size_t>(n) * A + a] = G > 0 ? best.i : 0;
        row_max[static_cast<size_t>(n) * A + a] = G > 0 ? best.v : 0.0;
    }
    __syncthreads();
    for (int g = tid; g < G; g += 256) {
        ArgMax c = wred[0][g];
        for (int w = 1; w < 4; ++w) c = am_combine(c, wred[w][g]);
        const size_t o = (static_cast<size_t>(n) * gridDim.x + blockIdx.x) * Gp + g;
        col_v[o] = c.nan ? NAN : c.v;
        col_i[o] = c.i;
    }
}

// grid N, 1024 threads: gt_argmax from the block partials, labels of
// utils/utils.py:176-188 and the ordered pos / neg index lists.
__global__ __launch_bounds__(1024) void at_label_kernel(
    int A, int Gp, int nblk, const int* __restrict__ gcount, const double* __restrict__ row_max,
    const double* __restrict__ col_v, const int* __restrict__ col_i, double neg_thr, double pos_thr,
    int32_t* __restrict__ row_arg, int8_t* __restrict__ label0, int* __restrict__ pos_list,
    int* __restrict__ neg_list, int* __restrict__ npos, int* __restrict__ nneg) {
    __shared__ int s_garg[kMaxG];
    const int n = blockIdx.x;
    const int G = gcount[n];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int g = tid; g < G; g += 1024) {
        // the block partials in order, eight loads in flight at a time (one round
        // trip per eight blocks, not per block); the fold order is unchanged
        ArgMax c{0.0, 0, 0};
        for (int b0 = 0; b0 < nblk; b0 += 8) {
            double vv[8];
            int ii[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const size_t o = (static_cast<size_t>(n) * nblk + min(b0 + u, nblk - 1)) * Gp + g;
                vv[u] = col_v[o];
                ii[u] = col_i[o];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (b0 + u < nblk) {
                    const ArgMax x{vv[u], ii[u], vv[u] != vv[u]};
                    c = b0 + u == 0 ? x : am_combine(c, x);
                }
            }
        }
        s_garg[g] = c.i;
    }
    __syncthreads();
    int8_t* lab = label0 + static_cast<size_t>(n) * A;
    const double* mx = row_max + static_cast<size_t>(n) * A;
    for (int a = tid; a < A; a += 1024) {
        int8_t l = -1;
        const double m = mx[a];
        if (m < neg_thr) l = 0;
        if (m >= pos_thr) l = 1;
        lab[a] = l;
    }
    __syncthreads();
    if (tid == 0) {
        int32_t* arg = row_arg + static_cast<size_t>(n) * A;
        for (int g = 0; g < G; ++g) {      // utils/utils.py:171-172 (later gt wins) and :187-188
            arg[s_garg[g]] = g;
            lab[s_garg[g]] = 1;
        }
    }
    __syncthreads();
    // ordered compaction of label==1 and label==0 positions: thread t counts its run
    // of anchors [t * per, (t + 1) * per), one block-wide exclusive scan of the
    // counts, then each thread writes its run in order (one barrier round, not one
    // per 1024 anchors)
    const int per = (A + 1023) / 1024;
    const int r0 = min(A, tid * per), r1 = min(A, r0 + per);
    int cp = 0, cn = 0;
    for (int a = r0; a < r1; ++a) {
        const int8_t l = lab[a];
        cp += l == 1;
        cn += l == 0;
    }
    long long both = static_cast<long long>(cp) | (static_cast<long long>(cn) << 32);  // (no carries: < 2^31 each)
    long long inc = both;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const long long u = __shfl_up(inc, d, 64);
        if (lane >= d) inc += u;
    }
    __shared__ long long s_wt[16];
    if (lane == 63) s_wt[wid] = inc;
    __syncthreads();
    long long pre = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
        const long long x = s_wt[w];
        if (w < wid) pre += x;
        tot += x;
    }
    const long long ex = pre + inc - both;
    int pp = static_cast<int>(ex & 0xffffffffll), pn = static_cast<int>(ex >> 32);
    int* pl = pos_list + static_cast<size_t>(n) * A;
    int* nl = neg_list + static_cast<size_t>(n) * A;
    for (int a = r0; a < r1; ++a) {
        const int8_t l = lab[a];
        if (l == 1) pl[pp++] = a;
        if (l == 0) nl[pn++] = a;
    }
    if (tid == 0) {
        npos[n] = static_cast<int>(tot & 0xffffffffll);
        nneg[n] = static_cast<int>(tot >> 32);
    }
}

// ------------------------------------------------------------- MT19937 wave
constexpr int kMtN = 624;
constexpr int kMtM = 397;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// numpy's rk_interval mask: all ones up to the highest set bit of v (v > 0)
__device__ __forceinline__ uint32_t mask_for(uint32_t v) {
    return v ? 0xffffffffu >> __builtin_clz(v) : 0u;
}
// mask_for(max(v, 1)): no zero test (for the walks' decision max(w & mask, 1) <=
// step, where a step <= 0 rejects whatever the mask)
__device__ __forceinline__ uint32_t mask_nz(uint32_t v) { return 0xffffffffu >> __builtin_clz(v | 1u); }

// ------------------------------------------------------------ stream walker
// The sampler kernels run as ONE 1024-thread workgroup: the MT19937 stream is a
// single sequential resource (image n's draws start where image n-1's ended).
//  * The raw state blocks live in an LDS ring of 3.  227 threads twist a block
//    from the previous one, each producing words t, t + 227, t + 454 in
//    registers (the one cross-thread input, the new word 0 that word 623
//    wraps to, is recomputed), so a block costs one barrier.
//  * The rejection automaton consumes the stream in windows of 1024 words,
//    thread t owning word t: word t's step is i_cur - #accepted(words < t),
//    accepted iff (w_t & mask(step)) <= step.  Each wave solves its 64 words
//    exactly for an assumed count of accepted words before it (ballot fixed
//    point), one barrier publishes the 16 wave counts, and the window is
//    settled when no count changed: the unique fixed point, since word t
//    depends only on words < t.  A word's decision depends on its step only
//    when (w & mask) lies that close to it, so guesses from the expected
//    acceptance rate settle in 2-3 rounds.
//  * Survivors / samples are read off the recorded swaps J (fy_final).
constexpr int kSampThreads = 1024;
constexpr int kSampWaves = kSampThreads / 64;
constexpr int kMaxKeep = 4096;  // recorded swaps / survivors per choice() call (LDS)
#ifdef FRCNN_SAMPLER_PROF
__device__ unsigned long long g_samp_prof[16];
#define SPROF_T0() const unsigned long long _t0 = __builtin_amdgcn_s_memtime()
#define SPROF_ADD(k, v) do { if (threadIdx.x == 0) g_samp_prof[k] += (v); } while (0)
#define SPROF_DT(k) SPROF_ADD(k, __builtin_amdgcn_s_memtime() - _t0)
#else
#define SPROF_T0() do {} while (0)
#define SPROF_ADD(k, v) do {} while (0)
#define SPROF_DT(k) do {} while (0)
#endif
// (windows of 2 / 4 chunks per wave measured 8 % / 32 % slower, 8 / 10 / 14 / 15 walking
// waves and sequential thresholds of 256 / 512 / 2048 steps lost too: profiles/r4_experiments.md)
constexpr int kWinWaves = 12;  // waves that walk a window; the others twist ahead
constexpr int kSubc = 1;       // 64-word chunks per walking wave and window
constexpr int kWinChunks = kWinWaves * kSubc;
constexpr int kWin = kWinChunks * 64;      // words per window
// a window (kWin words from pos <= 624) spans <= (624 + kWin - 1) / 624 + 1 blocks, + 1 being twisted
constexpr int kRing = (kMtN + kWin - 1) / kMtN + 2;
constexpr int kSeqBelow = 1024;  // steps below which one wave walks the window
static_assert(kSeqBelow <= (1 << 15), "the sequential walk's 16-bit fixed-point guess");

struct Stream {  // block-uniform: every thread tracks the same values
    int slot;    // ring slot of the block numpy's key[] holds
    int off;     // numpy's pos within it (0..624)
    int ngen;    // blocks twisted ahead of it (0..2)
};

struct WalkLds {
    uint32_t ring[kRing][kMtN];   // raw state blocks (the twist's input, the state handed back)
    uint32_t tring[kRing][kMtN];  // the same words tempered (what the walkers read)
    int4 rec[2][kSampWaves];  // per wave, by round parity: (accepted words, margin down, margin up, base)
    int last[kSampWaves];     // per wave: highest accepted word + 1 (the window that ends a call)
    int seq[2][2];            // one-wave walk, by window parity: (step left, words used)
};

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// numpy's mt19937_gen: nw = the state block after old (words i < 227 read
// old[i + 397], later words the new word 227 before them; word 623 reads the
// new word 0).  Threads t = 0..226 of the caller's group do the work.
__device__ __forceinline__ void mt_twist(const uint32_t* __restrict__ old, uint32_t* __restrict__ nw,
                                         uint32_t* __restrict__ tw, int t) {
    if (t < kMtN - kMtM) {
        const uint32_t a = old[t + kMtM] ^ mt_mix(old[t], old[t + 1]);
        const uint32_t b = a ^ mt_mix(old[t + 227], old[t + 228]);
        nw[t] = a;
        nw[t + 227] = b;
        tw[t] = mt_temper(a);
        tw[t + 227] = mt_temper(b);
        if (t + 454 < kMtN - 1) {
            const uint32_t c = b ^ mt_mix(old[t + 454], old[t + 455]);
            nw[t + 454] = c;
            tw[t + 454] = mt_temper(c);
        } else if (t + 454 == kMtN - 1) {
            const uint32_t n0 = old[kMtM] ^ mt_mix(old[0], old[1]);
            const uint32_t c = b ^ mt_mix(old[kMtN - 1], n0);
            nw[kMtN - 1] = c;
            tw[kMtN - 1] = mt_temper(c);
        }
    }
}

__device__ __forceinline__ void stream_load(WalkLds& S, Stream& st, const uint32_t* __restrict__ rng) {
    for (int i = threadIdx.x; i < kMtN; i += kSampThreads) {
        const uint32_t v = rng[i];
        S.ring[0][i] = v;
        S.tring[0][i] = mt_temper(v);
    }
    st.slot = 0;
    st.off = static_cast<int>(rng[kMtN]);
    st.ngen = 0;
}

__device__ __forceinline__ void stream_store(const WalkLds& S, const Stream& st, uint32_t* __restrict__ rng) {
    for (int i = threadIdx.x; i < kMtN; i += kSampThreads) rng[i] = S.ring[st.slot][i];
    if (threadIdx.x == 0) rng[kMtN] = static_cast<uint32_t>(st.off);
}

// Tempered word `off` past the stream position: the ring's blocks are contiguous in
// LDS, so the word sits at (slot * 624 + pos + off) modulo the ring (pos + off
// < 624 + kWin keeps the sum below twice the ring: one conditional subtract).
static_assert(kWin <= kRing * kMtN, "ring_word: one conditional subtract must wrap any window word");
__device__ __forceinline__ uint32_t ring_word(const WalkLds& S, const Stream& st, int off) {
    int f = st.slot * kMtN + st.off + off;
    f -= f >= kRing * kMtN ? kRing * kMtN : 0;
    return (&S.tring[0][0])[f];
}

// Fisher-Yates steps i = i_hi .. 1 of one choice() call on the stream; for
// steps i >= rec_lo, J[i - rec_lo] = j.  Block-uniform; ends with a barrier.
// Inclusive prefix sum over each row of 16 lanes (DPP row shifts).
__device__ __forceinline__ int row16_scan_add(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
    return x;
}

// Both margins of a wave in one reduction: dn and up (clamped to 16 bits; a
// clamped margin only makes the check conservative) packed, v_pk_min_u16 over
// DPP row shifts, the four row minima combined on the scalar unit.
typedef unsigned short __attribute__((ext_vector_type(2))) u16x2;
__device__ __forceinline__ uint32_t pk_min16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ void wave_min2(uint32_t& dn, uint32_t& up) {
    uint32_t x = (min(dn, 0xffffu) << 16) | min(up, 0xffffu);
    x = pk_min16(x, __builtin_amdgcn_update_dpp(0xffffffffu, x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = pk_min16(x, __builtin_amdgcn_update_dpp(0xffffffffu, x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = pk_min16(x, __builtin_amdgcn_update_dpp(0xffffffffu, x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = pk_min16(x, __builtin_amdgcn_update_dpp(0xffffffffu, x, 0x118, 0xf, 0xf, false));  // row_shr:8
    const uint32_t r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31);
    const uint32_t r2 = __builtin_amdgcn_readlane(x, 47), r3 = __builtin_amdgcn_readlane(x, 63);
    dn = min(min(r0 >> 16, r1 >> 16), min(r2 >> 16, r3 >> 16));
    up = min(min(r0 & 0xffffu, r1 & 0xffffu), min(r2 & 0xffffu, r3 & 0xffffu));
}

__device__ void fy_walk(WalkLds& S, Stream& st, int i_hi, int rec_lo, int* J) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int i_cur = i_hi;
    // S.rec's buffer parity runs on across windows: a wave reading the last round's
    // counts of one window and a wave publishing the next window's first round use
    // different buffers, so a window needs no closing barrier (its round barriers
    // order the ring-word reads before the next twists)
    int par = 0;
    while (i_cur >= 1) {
        const int need = (st.off + kWin - 1) / kMtN;  // blocks past st.slot this window reaches
        {
            SPROF_T0();
            while (st.ngen < need) {  // (only when the twisting waves fell behind)
                mt_twist(S.ring[(st.slot + st.ngen) % kRing], S.ring[(st.slot + st.ngen + 1) % kRing],
                         S.tring[(st.slot + st.ngen + 1) % kRing], tid);
                __syncthreads();
                ++st.ngen;
                SPROF_ADD(1, 1);
            }
            SPROF_DT(2);
        }
        // waves kWinWaves.. twist the next block into a free ring slot while the
        // others walk the window; the window's barriers publish it
        const bool gen = st.ngen < kRing - 1;
        if (gen && wid >= kWinWaves)
            for (int t = tid - kWinWaves * 64; t < kMtN - kMtM; t += (kSampWaves - kWinWaves) * 64)
                mt_twist(S.ring[(st.slot + st.ngen) % kRing], S.ring[(st.slot + st.ngen + 1) % kRing],
                         S.tring[(st.slot + st.ngen + 1) % kRing], t);
        SPROF_ADD(0, 1);
        SPROF_T0();
        if (i_cur < kSeqBelow) {
            // Small calls (narrow masks: a word's decision is sensitive to its exact
            // step, so the parallel rounds cascade): wave 0 walks the window's 64-word
            // chunks in order, each solved exactly on the known step.
            if (wid == 0) {
                int i_loc = i_cur, used = 0;
                auto word = [&](int c) { return ring_word(S, st, 64 * c + lane); };  // chunk c's word
                uint32_t wn = word(0);  // the next chunk's word is read during this one's fixed point
                for (int c = 0; c < kWinChunks && i_loc >= 1; ++c) {
                    const uint32_t wc = wn;
                    if (c + 1 < kWinChunks) wn = word(c + 1);
                    // (a guess: any start reaches the same fixed point) the expected
                    // acceptances before the lane, (i + 1) / 2^bits(i) per word, in
                    // 16-bit fixed point (i < kSeqBelow here)
                    const uint32_t pa16 = (static_cast<uint32_t>(i_loc + 1) << 16) >>
                                          (32 - __builtin_clz(static_cast<uint32_t>(i_loc)));
                    const int ig0 = i_loc - static_cast<int>((static_cast<uint32_t>(lane) * pa16) >> 16);
                    const uint32_t ig0p = static_cast<uint32_t>(ig0 > 0 ? ig0 : 0);
                    uint64_t ac = __builtin_amdgcn_ballot_w64(max(wc & mask_nz(ig0p), 1u) <= ig0p);
                    int ilc;
                    uint32_t mc;
                    for (;;) {
                        const int below = static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                            static_cast<uint32_t>(ac >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(ac), 0u)));
                        ilc = i_loc - below;
                        // accepted iff ilc >= 1 and (w & mask) <= ilc, i.e.
                        // max(w & mask, 1) <= max(ilc, 0): one compare feeds the ballot
                        const uint32_t ip = static_cast<uint32_t>(ilc > 0 ? ilc : 0);
                        mc = mask_nz(ip);
                        const uint64_t nac = __builtin_amdgcn_ballot_w64(max(wc & mc, 1u) <= ip);
                        if (nac == ac) break;
                        ac = nac;
                    }
                    if (i_loc >= rec_lo && ((ac >> lane) & 1ull) && ilc >= rec_lo)  // (i_loc: wave-uniform skip)
                        J[ilc - rec_lo] = static_cast<int>(wc & mc);
                    const int cntc = __popcll(ac);
                    used = i_loc - cntc < 1 ? 64 * c + 64 - __clzll(ac) : 64 * (c + 1);
                    i_loc -= cntc;
                    SPROF_ADD(9, 1);
                }
                if (lane == 0) {  // (double-buffered by the parity: no closing barrier)
                    S.seq[par & 1][0] = i_loc;
                    S.seq[par & 1][1] = used;
                }
            }
            __syncthreads();
            SPROF_DT(10);
            const int i_new = S.seq[par & 1][0], consumed = S.seq[par & 1][1];
            par ^= 1;
            i_cur = i_new;
            if (gen) ++st.ngen;
            st.off += consumed;
            while (st.off > kMtN) {
                st.off -= kMtN;
                st.slot = (st.slot + 1) % kRing;
                --st.ngen;
            }
            continue;
        }
        // wave wid walks chunks wid * kSubc .. + kSubc - 1 (64 words each, in
        // stream order); its fixed point runs over all of them (Gauss-Seidel:
        // each chunk's steps from the counts of the chunks before it)
        uint32_t w[kSubc];
#pragma unroll
        for (int sc = 0; sc < kSubc; ++sc) {
            w[sc] = ring_word(S, st, wid < kWinWaves ? (wid * kSubc + sc) * 64 + lane : 0);
        }
        const float p_acc = (static_cast<float>(i_cur) + 1.0f) *
                            __builtin_amdgcn_rcpf(static_cast<float>(mask_for(static_cast<uint32_t>(i_cur))) + 1.0f);
        auto guess = [&](int v) { return static_cast<int>(static_cast<float>(v * 64) * p_acc); };
        int base = guess(wid * kSubc);
        uint64_t acc[kSubc];
#pragma unroll
        for (int sc = 0; sc < kSubc; ++sc) {
            const int ig = i_cur - base - static_cast<int>(static_cast<float>(sc * 64 + lane) * p_acc);
            const uint32_t igp = static_cast<uint32_t>(ig > 0 ? ig : 0);
            acc[sc] = __builtin_amdgcn_ballot_w64(max(w[sc] & mask_nz(igp), 1u) <= igp);
        }
        // Round: each unsettled wave solves its words for its assumed base and
        // publishes (count, margins, base): its pattern stays exact for any base in
        // [base - up, base + down] (no word changes its decision or mask width).
        // The first wave whose exact base (prefix of the counts before it) falls
        // outside its margins, and every wave after it, re-solves next round with
        // the new prefix; the waves before it are settled.  Counts hardly depend on
        // the base, so the first round's guesses are usually inside the margins and
        // the rest settle in the second; each round settles at least one more wave.
        int il[kSubc], total = 0;
        uint32_t m[kSubc];
        bool a[kSubc];
#pragma unroll
        for (int sc = 0; sc < kSubc; ++sc) {
            il[sc] = 0;
            m[sc] = 0;
            a[sc] = false;
        }
        bool done = wid >= kWinWaves;  // the twisting waves only keep the barriers
        for (;;) {  // rounds
            if (!done) {
                for (;;) {  // this wave's words, exact for the assumed `base`
                    bool ch = false;
                    int pre = 0;
#pragma unroll
                    for (int sc = 0; sc < kSubc; ++sc) {
                        const int below = pre + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                            static_cast<uint32_t>(acc[sc] >> 32),
                            __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(acc[sc]), 0u)));
                        il[sc] = i_cur - base - below;
                        // accepted iff il >= 1 and (w & mask) <= il, i.e.
                        // max(w & mask, 1) <= max(il, 0): one compare feeds the ballot
                        // (the lane's decision is read back from it after the loop)
                        const uint32_t ip = static_cast<uint32_t>(il[sc] > 0 ? il[sc] : 0);
                        m[sc] = mask_nz(ip);
                        const uint64_t nacc = __builtin_amdgcn_ballot_w64(max(w[sc] & m[sc], 1u) <= ip);
                        ch |= nacc != acc[sc];
                        acc[sc] = nacc;
                        pre += __popcll(nacc);
                    }
                    if (!ch) break;
                }
            }
            // Margins from the first round on: a wave's pattern depends on its
            // base only where (w & mask) lies that close to the step, so at wide
            // masks the guessed bases usually fall inside the margins and the window
            // settles in one round (settled waves keep d == 0 and need none).
            uint32_t dn = 0, up = 0;
            int cnt = 0;
#pragma unroll
            for (int sc = 0; sc < kSubc; ++sc) {
                cnt += __popcll(acc[sc]);
                a[sc] = (acc[sc] >> lane) & 1ull;
            }
            if (!done) {
                dn = up = 0x3fffffffu;
#pragma unroll
                for (int sc = 0; sc < kSubc; ++sc) {
                    uint32_t dns, ups;
                    if (il[sc] < 1) {
                        dns = 0x3fffffffu;
                        ups = static_cast<uint32_t>(-il[sc]);
                    } else {
                        const uint32_t lo = (m[sc] >> 1) + 1u;  // 2^k of the mask m = 2^(k+1) - 1
                        const uint32_t v = w[sc] & m[sc];
                        const uint32_t u = static_cast<uint32_t>(il[sc]);
                        dns = a[sc] ? u - (v > lo ? v : lo) : u - lo;
                        ups = a[sc] ? m[sc] - u : v - 1u - u;
                    }
                    dn = dns < dn ? dns : dn;
                    up = ups < up ? ups : up;
                }
                wave_min2(dn, up);
            }
            if (lane == 0 && wid < kWinWaves)
                S.rec[par][wid] = make_int4(cnt, static_cast<int>(dn), static_cast<int>(up), base);
            __syncthreads();
            const int4 r = lane < kWinWaves ? S.rec[par][lane] : make_int4(0, 0, 0, 0);
            const int incl = row16_scan_add(r.x);  // lanes 0..15: prefix over waves
            const int excl = incl - r.x;
            const int d = excl - r.w;  // exact base - assumed base of wave `lane`
            const uint64_t bad = __builtin_amdgcn_ballot_w64(lane < kWinWaves && (d > r.y || -d > r.z));
            const int first_bad = bad ? __ffsll(static_cast<unsigned long long>(bad)) - 1 : kWinWaves;
            const int my_excl = __builtin_amdgcn_readlane(excl, wid < kWinWaves ? wid : 0);
            if (wid < first_bad) {
                if (!done) {  // settled: same pattern at the exact base, steps shifted
#pragma unroll
                    for (int sc = 0; sc < kSubc; ++sc) il[sc] -= my_excl - base;
                    base = my_excl;
                    done = true;
                }
            } else {
                base = my_excl;
            }
            total = __builtin_amdgcn_readlane(incl, kWinWaves - 1);
            par ^= 1;
            SPROF_ADD(3, 1);
            if (first_bad == kWinWaves) break;
        }
        SPROF_DT(4);
        if (i_cur - base >= rec_lo) {  // (the wave's first step: a wave-uniform skip)
#pragma unroll
            for (int sc = 0; sc < kSubc; ++sc)
                if (a[sc] && il[sc] >= rec_lo) J[il[sc] - rec_lo] = static_cast<int>(w[sc] & m[sc]);
        }
        int consumed = kWin;
        if (i_cur - total < 1) {  // the call ends inside this window
            if (lane == 0 && wid < kWinWaves) {
                int last = 0;
#pragma unroll
                for (int sc = 0; sc < kSubc; ++sc)
                    if (acc[sc]) last = 64 * (wid * kSubc + sc) + 64 - __clzll(acc[sc]);
                S.last[wid] = last;
            }
            __syncthreads();
            consumed = static_cast<int>(__ockl_wfred_max_u32(lane < kWinWaves ? static_cast<uint32_t>(S.last[lane]) : 0u));
        }
        i_cur -= total;
        if (gen) ++st.ngen;
        st.off += consumed;
        while (st.off > kMtN) {  // pos == 624 stays in its block, like numpy
            st.off -= kMtN;
            st.slot = (st.slot + 1) % kRing;
            --st.ngen;
        }
    }
    __syncthreads();  // the call's swap records (J) and S.last are read next
}

// Final values at permutation positions [p_lo, p_hi) of the cnt-element
// shuffle whose swaps J[i - rec_lo] are recorded for steps i >= rec_lo
// (p_lo >= rec_lo, or p_lo == 0 with rec_lo == 1).  Tracing backwards in
// time: position p takes, at step p, the value position J[p] holds then, and
// position x's value before step t is the one position i* held before step i*,
// i* = min{i > t : J[i] == x} (its last swap), or x itself.  So
//   v(p) = chase(J[p], X[p]),   X[p] = min{i > p : J[i] == J[p]},
//   chase(x, i): while i exists: x = i, i = F[i],   F[v] = min{i > v : J[i] == v}.
// F (atomicMin, indexed from p_lo) and the steps bucketed by value (1024
// buckets of 16, value & 1023) live in LDS; X[p] is the smallest bucket entry
// past p with p's value (a full scan of J when the bucket overflowed: value v
// recurs ~ln(cnt / v) times, so only the smallest values come close).
constexpr int kBuckets = 1024;
constexpr int kBucketCap = 16;
struct FinalLds {
    int F[kMaxKeep];
    int bcnt[kBuckets];
    int bkt[kBuckets][kBucketCap];
};

template <class Emit>
__device__ void fy_final(int cnt, int rec_lo, int p_lo, int p_hi, const int* J, FinalLds& L, Emit emit) {
    const int tid = threadIdx.x;
    SPROF_T0();
    const int f0 = p_lo;  // every chased index is >= p_lo (p_lo == 0 only when rec_lo == 1)
    constexpr int kNone = 0x7fffffff;
    for (int v = f0 + tid; v < cnt; v += kSampThreads) L.F[v - f0] = kNone;
    for (int b = tid; b < kBuckets; b += kSampThreads) L.bcnt[b] = 0;
    __syncthreads();
    const int q0 = max(p_lo, 1);  // positions with a first query X[p]
    for (int i = rec_lo + tid; i < cnt; i += kSampThreads) {
        const int v = J[i - rec_lo];
        if (v < i && v >= f0) atomicMin(&L.F[v - f0], i);
        if (i > q0) {
            const int b = v & (kBuckets - 1);
            const int slot = atomicAdd(&L.bcnt[b], 1);
            if (slot < kBucketCap) L.bkt[b][slot] = i;
        }
    }
    __syncthreads();
    for (int p = p_lo + tid; p < p_hi; p += kSampThreads) {
        int x = 0, i;
        if (p == 0) {
            i = L.F[0];
        } else {
            x = J[p - rec_lo];
            const int b = x & (kBuckets - 1);
            const int n = L.bcnt[b];
            i = kNone;
            if (n <= kBucketCap) {
                for (int s = 0; s < n; ++s) {
                    const int t = L.bkt[b][s];
                    if (t > p && t < i && J[t - rec_lo] == x) i = t;
                }
            } else {
                for (int t = p + 1; t < cnt; ++t)
                    if (J[t - rec_lo] == x) {
                        i = t;
                        break;
                    }
            }
        }
        while (i < cnt) {
            x = i;
            i = L.F[i - f0];
        }
        emit(p, x);
    }
    __syncthreads();
    SPROF_DT(5);
}

// ---------------------------------------------------------- AnchorTarget RNG
// One workgroup: for each image in order, the two choice() calls of
// utils/utils.py:190-202.  Kept anchors are marked in keep[n][a] (zeroed by
// the caller); pos_sampled / neg_sampled record whether a call happened.

__device__ void at_draws(WalkLds& S, Stream& st, int* J, int N, int n_sample, int n_pos_max,
                         const int* __restrict__ npos, const int* __restrict__ nneg, int* __restrict__ sampled,
                         int4* __restrict__ calls, int* __restrict__ jrec) {
    for (int n = 0; n < N; ++n) {
        const int P = npos[n];
        const int Q = nneg[n];
        const int pos_after = P > n_pos_max ? n_pos_max : P;
        const int neg_keep = n_sample - pos_after;
        for (int call = 0; call < 2; ++call) {
            const int cnt = call == 0 ? P : Q;
            const int m = call == 0 ? n_pos_max : neg_keep;  // survivors
            const bool do_call = cnt > m;
            const int k = cnt - m;  // disabled = perm[:k]; survivors = perm[k:]
            if (threadIdx.x == 0) {
                sampled[2 * n + call] = do_call ? 1 : 0;
                calls[2 * n + call] = do_call ? make_int4(cnt, k, cnt, 0) : make_int4(0, 0, 0, 0);
            }
            if (!do_call) continue;
            fy_walk(S, st, cnt - 1, k, J);
            SPROF_ADD(7, cnt);
            // the swaps of the recorded steps; the survivors are read off them by
            // samp_emit_kernel (no RNG: off the draws' stream)
            int* jg = jrec + static_cast<size_t>(2 * n + call) * kMaxKeep;
            for (int i = threadIdx.x; i < cnt - k; i += kSampThreads) jg[i] = J[i];
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(kSampThreads) void at_sample_kernel(
    int N, int A, int n_sample, int n_pos_max, const int* __restrict__ pos_list,
    const int* __restrict__ neg_list, const int* __restrict__ npos, const int* __restrict__ nneg,
    uint32_t* __restrict__ rng, int* __restrict__ sampled, int4* __restrict__ calls, int* __restrict__ jrec,
    const int* __restrict__ gate) {
    __shared__ WalkLds S;
    __shared__ int J[kMaxKeep];
    if (gate && *gate == 0) return;  // the chip-wide draws succeeded (draw_chain_kernel)
    SPROF_T0();
    Stream st;
    stream_load(S, st, rng);
    __syncthreads();
    at_draws(S, st, J, N, n_sample, n_pos_max, npos, nneg, sampled, calls, jrec);
    stream_store(S, st, rng);
    SPROF_DT(6);
}

// grid (ceil(A/256), N): final label (after disabling) and regression target
// bbox2reg(anchor, bbox[argmax]) (utils/utils.py:75-100,146-150; anchor stats
// fp32, box stats fp64).
__global__ __launch_bounds__(256) void at_finish_kernel(
    const float* __restrict__ anchors, int A, const double* __restrict__ gt,
    const int* __restrict__ gcount, int Gp, const int32_t* __restrict__ row_arg,
    const int8_t* __restrict__ label0, const uint8_t* __restrict__ keep,
    const int* __restrict__ sampled, int32_t* __restrict__ label, double* __restrict__ reg) {
    const int n = blockIdx.y;
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    const size_t o = static_cast<size_t>(n) * A + a;
    const int8_t l0 = label0[o];
    int32_t l = -1;
    if (l0 == 1) l = (!sampled[2 * n] || keep[o]) ? 1 : -1;
    else if (l0 == 0) l = (!sampled[2 * n + 1] || keep[o]) ? 0 : -1;
    label[o] = l;
    const int G = gcount[n];
    double* r = reg + o * 4;
    if (G == 0) {
        r[0] = r[1] = r[2] = r[3] = 0.0;
        return;
    }
    const float* an = anchors + static_cast<size_t>(a) * 4;
    const double* b = gt + (static_cast<size_t>(n) * Gp + row_arg[o]) * 4;
    const float ah = an[2] - an[0];
    const float aw = an[3] - an[1];
    const float acx = (an[2] + an[0]) / 2.0f;
    const float acy = (an[1] + an[3]) / 2.0f;
    const double bh = b[2] - b[0];
    const double bw = b[3] - b[1];
    const double bcx = (b[2] + b[0]) / 2.0;
    const double bcy = (b[1] + b[3]) / 2.0;
    r[0] = (bcx - static_cast<double>(acx)) / static_cast<double>(ah);
    r[1] = (bcy - static_cast<double>(acy)) / static_cast<double>(aw);
    r[2] = log(bh / static_cast<double>(ah));
    r[3] = log(bw / static_cast<double>(aw));
}

// ----------------------------------------------------- ProposalTarget (f64)
// grid N, 1024 threads: roi_all = concat(roi fp32 -> fp64, gt), IoU with the gt,
// row argmax / max, label of the assigned gt, ordered pos / neg lists
// (utils/utils.py:229-258).
__global__ __launch_bounds__(1024) void pt_iou_kernel(
    const float* __restrict__ rois, const int* __restrict__ rcount, int Rp,
    const double* __restrict__ gt, const double* __restrict__ gl, const int* __restrict__ gcount,
    int Gp, double pos_thr, double neg_hi, double neg_lo, double* __restrict__ roi_all,
    int32_t* __restrict__ assign, int* __restrict__ pos_list, int* __restrict__ neg_list,
    int* __restrict__ npos, int* __restrict__ nneg) {
    __shared__ double sg[kMaxG][4];
    __shared__ double sa[kMaxG];
    __shared__ int s_w[16];
    const int n = blockIdx.x;
    const int G = gcount[n];
    const int Rn = rcount[n];
    const int T = Rn + G;
    const int stride = Rp + Gp;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int g = tid; g < G; g += 1024) {
        for (int c = 0; c < 4; ++c) sg[g][c] = gt[(static_cast<size_t>(n) * Gp + g) * 4 + c];
        sa[g] = area_np(sg[g]);
    }
    __syncthreads();
    int pbase = 0, nbase = 0;
    for (int t0 = 0; t0 < T; t0 += 1024) {
        const int t = t0 + tid;
        bool isp = false, isn = false;
        if (t < T) {
            double box[4];
            for (int c = 0; c < 4; ++c)
                box[c] = t < Rn ? static_cast<double>(rois[(static_cast<size_t>(n) * Rp + t) * 4 + c])
                                : sg[t - Rn][c];
            for (int c = 0; c < 4; ++c) roi_all[(static_cast<size_t>(n) * stride + t) * 4 + c] = box[c];
            const double ab = area_np(box);
            double best = 0.0;
            int bi = 0;
            bool bnan = false;
            for (int g = 0; g < G; ++g) {
                const double v = iou_np(box, ab, sg[g], sa[g]);
                if (g == 0) {
                    best = v;
                    bnan = v != v;
                } else if (np_better(v, best, bnan)) {
                    best = v;
                    bi = g;
                    bnan = v != v;
                }
            }
            if (G == 0) best = 0.0;
            assign[static_cast<size_t>(n) * stride + t] = bi;
            isp = best >= pos_thr;
            isn = best < neg_hi && best >= neg_lo;
        }
        const uint64_t bp = __ballot(isp), bn = __ballot(isn);
        if (lane == 0) s_w[wid] = __popcll(bp) | (__popcll(bn) << 16);
        __syncthreads();
        int bpp = 0, bnn = 0, tp = 0, tn = 0;
        for (int w = 0; w < 16; ++w) {
            const int v = s_w[w];
            if (w < wid) {
                bpp += v & 0xffff;
                bnn += v >> 16;
            }
            tp += v & 0xffff;
            tn += v >> 16;
        }
        if (isp) pos_list[static_cast<size_t>(n) * stride + pbase + bpp + __popcll(bp & lanemask_lt())] = t;
        if (isn) neg_list[static_cast<size_t>(n) * stride + nbase + bnn + __popcll(bn & lanemask_lt())] = t;
        pbase += tp;
        nbase += tn;
        __syncthreads();
    }
    if (tid == 0) {
        npos[n] = pbase;
        nneg[n] = nbase;
    }
}

// One workgroup: the two choice() calls of utils/utils.py:248-258 per image,
// in image order; sample order = pos perm prefix, then neg perm prefix.
__device__ void pt_draws(WalkLds& S, Stream& st, int* J, int N, int n_sample, int pos_per_image,
                         const int* __restrict__ npos, const int* __restrict__ nneg, int* __restrict__ scount,
                         int* __restrict__ spos, int4* __restrict__ calls, int* __restrict__ jrec) {
    for (int n = 0; n < N; ++n) {
        const int P = npos[n], Q = nneg[n];
        const int kp = P < pos_per_image ? P : pos_per_image;
        int kn = n_sample - kp;
        kn = Q < kn ? Q : kn;
        for (int call = 0; call < 2; ++call) {
            const int cnt = call == 0 ? P : Q;
            const int k = call == 0 ? kp : kn;
            const int off = call == 0 ? 0 : kp;
            if (threadIdx.x == 0) calls[2 * n + call] = cnt > 0 ? make_int4(cnt, 1, k, off) : make_int4(0, 0, 0, 0);
            if (cnt == 0) continue;
            fy_walk(S, st, cnt - 1, 1, J);  // every step: J[i - 1]
            int* jg = jrec + static_cast<size_t>(2 * n + call) * kMaxKeep;  // read by samp_emit_kernel
            for (int i = threadIdx.x; i < cnt - 1; i += kSampThreads) jg[i] = J[i];
            __syncthreads();
            SPROF_ADD(8, 1);
        }
        if (threadIdx.x == 0) {
            scount[n] = kp + kn;
            spos[n] = kp;
        }
    }
}

__global__ __launch_bounds__(kSampThreads) void pt_sample_kernel(
    int N, int stride, int n_sample, int pos_per_image, const int* __restrict__ pos_list,
    const int* __restrict__ neg_list, const int* __restrict__ npos, const int* __restrict__ nneg,
    uint32_t* __restrict__ rng, int* __restrict__ scount,
    int* __restrict__ spos, int4* __restrict__ calls, int* __restrict__ jrec, const int* __restrict__ gate) {
    __shared__ WalkLds S;
    __shared__ int J[kMaxKeep];
    if (gate && *gate == 0) return;  // the chip-wide draws succeeded (draw_chain_kernel)
    Stream st;
    stream_load(S, st, rng);
    __syncthreads();
    pt_draws(S, st, J, N, n_sample, pos_per_image, npos, nneg, scount, spos, calls, jrec);
    stream_store(S, st, rng);
}

// Both creators' serial draws in one launch (the walk behind frcnn_target_draws'
// chip-wide pass: one gate check, one workgroup waiting for its LDS, not two).
__global__ __launch_bounds__(kSampThreads) void target_sample_kernel(
    int n_at, int at_n_sample, int at_pos_max, const int* __restrict__ at_npos, const int* __restrict__ at_nneg,
    int* __restrict__ at_sampled, int4* __restrict__ at_calls, int* __restrict__ at_jrec, int n_pt,
    int pt_n_sample, int pt_pos_per_image, const int* __restrict__ pt_npos, const int* __restrict__ pt_nneg,
    int* __restrict__ pt_scount, int* __restrict__ pt_spos, int4* __restrict__ pt_calls,
    int* __restrict__ pt_jrec, uint32_t* __restrict__ rng, const int* __restrict__ gate) {
    __shared__ WalkLds S;
    __shared__ int J[kMaxKeep];
    if (gate && *gate == 0) return;
    Stream st;
    stream_load(S, st, rng);
    __syncthreads();
    at_draws(S, st, J, n_at, at_n_sample, at_pos_max, at_npos, at_nneg, at_sampled, at_calls, at_jrec);
    pt_draws(S, st, J, n_pt, pt_n_sample, pt_pos_per_image, pt_npos, pt_nneg, pt_scount, pt_spos, pt_calls, pt_jrec);
    stream_store(S, st, rng);
}

// One workgroup per choice() call (b = 2 image + call): the positions the
// caller needs, read off the recorded swaps the sampler left in jrec (fy_final;
// no RNG, so on any stream after the draws).  AnchorTarget (kMode 0) marks the
// survivors perm[k:] in keep; ProposalTarget (1) writes the sample perm[:k] in order.
template <int kMode>
__global__ __launch_bounds__(kSampThreads) void samp_emit_kernel(const int4* __restrict__ calls,
                                                                 const int* __restrict__ jrec,
                                                                 const int* __restrict__ pos_list,
                                                                 const int* __restrict__ neg_list, int stride,
                                                                 uint8_t* __restrict__ keep,
                                                                 int* __restrict__ sample, int n_sample) {
    __shared__ int Jl[kMaxKeep];
    __shared__ FinalLds FL;
    const int b = blockIdx.x;
    const int4 c = calls[b];  // cnt (0: no call), lowest recorded step, p_hi, output offset
    if (c.x == 0) return;
    const int cnt = c.x, rlo = c.y;
    const int jn = cnt - rlo > 0 ? cnt - rlo : 0;
    const int* jg = jrec + static_cast<size_t>(b) * kMaxKeep;
    for (int i = threadIdx.x; i < jn; i += kSampThreads) Jl[i] = jg[i];
    __syncthreads();
    const int n = b >> 1;
    const int* lst = ((b & 1) ? neg_list : pos_list) + static_cast<size_t>(n) * stride;
    if (kMode == 0) {
        uint8_t* kp = keep + static_cast<size_t>(n) * stride;
        fy_final(cnt, rlo, rlo, cnt, Jl, FL, [&](int, int v) { kp[lst[v]] = 1; });  // rlo >= 1
    } else {
        int* out = sample + static_cast<size_t>(n) * n_sample + c.w;
        fy_final(cnt, rlo, 0, c.z, Jl, FL, [&](int p, int v) { out[p] = lst[v]; });
    }
}

// ========================================================= chip-wide draws
// The draws of at_sample_kernel / pt_sample_kernel (one MT19937 stream, every
// choice() call of every image in order), spread over the chip.  The walk's
// state between words is (q, K): q words consumed, K steps accepted; the
// calls' bounds are a function of K alone (walk c runs bounds hi_c .. 1 while
// K is in [cum[c] - hi_c, cum[c])), so a stretch of words maps each entering K
// to a leaving K.  The stream is cut into segments of seg_l words (1024, or 256 for short streams) and, for
// every segment, that map is tabulated over the K's the walk can plausibly
// hold at the segment's start -- the domain: the expected K from the calls'
// mask regions (E[words per step] = (mask + 1) / (bound + 1)) +- mult sigma --
// one lane per entering K (draw_table_kernel, chip-wide; a lane's walk is three
// VALU per word, the mask and the call refreshed only at the wave's nearest
// region or call edge).  Tables are composed over groups of kGrpG segments
// (draw_group_kernel) and chained over the groups (draw_chain_kernel): the
// exact K at every segment start.  Segments holding a recorded swap or the
// stream's last draw are then walked exactly, one wave each
// (draw_record_kernel).  A K outside a domain or a plan over the workspace's
// capacity sets hdr.fail and the serial sampler, gated on it, does the draws:
// exact either way (the words, bounds and acceptance rule are the serial
// walk's; only the order of evaluation differs).
constexpr int kSegLMax = 1024;       // words per segment: 1024, or 256 for short streams
constexpr int kGrpG = 16;            // segments per group
constexpr int kDrawWalks = 256;      // calls with >= 1 step (N <= 128 images)
constexpr int kDrawDcap = 4096;      // entering K's per segment
constexpr int kDrawSegMax = 1024;    // segments (1 M words)
constexpr int kDrawHiMax = 65535;    // bounds < 2^16: <= 16 mask regions per call
constexpr int kDrawPieces = kDrawWalks * 16;
constexpr int kChainLds = 65536;     // composite entries draw_chain_kernel stages in LDS
constexpr uint16_t kMiss = 0xffffu;  // a leaving K outside the next segment's domain
static_assert(kGrpG * kDrawDcap * 2 <= 128 * 1024, "a group's tables fit draw_group_kernel's LDS");
static_assert(kDrawSegMax <= 1024 && 2 * kDrawWalks / 2 <= 1024, "one thread per segment / call in the setup");

struct DrawHdr {
    int fail;  // 0: the chip-wide draws hold; 1: plan over capacity; 2: a K left its domain
    int nw, ktot, nseg, ngrp, nblk, off0, dmax;
    int miss;   // the group whose composite missed (fail 2), else -1
    int seg_l;  // words per segment
};

struct DrawCap {
    int smax, nbmax, tabmax, premax;  // smax == 0: the serial sampler only
};

struct DrawBufs {
    DrawHdr* hdr;
    int* w_hi;    // [kDrawWalks] walk c: bounds hi_c .. 1
    int* w_cum;   // [kDrawWalks] K after walk c
    int* w_rec;   // [kDrawWalks] lowest recorded bound
    int* w_row;   // [kDrawWalks] jrec row (the choice() call)
    int* s_lo;    // [smax + 1] segment s's domain: entering K in [s_lo, s_lo + s_d)
    int* s_d;     // [smax + 1]
    int* s_toff;  // [smax + 1] table offsets (prefix of s_d)
    int* s_item;  // [smax + 1] prefix of ceil(s_d / 256): a workgroup per 256 entering K's
    int* g_poff;  // [smax / kGrpG + 2] group prefix-table offsets
    int* kseg;    // [smax + 1] exact K at each segment start
    uint16_t* tab;  // per segment, per entering K: leaving K - s_lo[s + 1] (kMiss outside)
    uint16_t* pre;  // per group, per segment j, per entering K of the group: K after j (rel.)
    uint32_t* raw;  // [nbmax][624] state blocks (block 0 = the key handed in)
    uint32_t* tw;   // the words tempered, from the draws' first: word q of the draws is tw[q]
};

template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}
// Inclusive scan of one value per thread over a 1024-thread block (sh: 16 slots).
template <class T>
__device__ T block_incl_scan(T v, T* sh, T& tot) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    v = wave_incl_scan(v);
    if (lane == 63) sh[wid] = v;
    __syncthreads();
    T pre = 0, all = 0;
    for (int i = 0; i < 16; ++i) {
        const T x = sh[i];
        if (i < wid) pre += x;
        all += x;
    }
    __syncthreads();
    tot = all;
    return v + pre;
}

// H(n) = sum 1/i and H2(n) = sum 1/i^2 (asymptotic past 32; the plan only
// centres the domains, it decides nothing)
struct HarmTab {
    double h1[65], h2[65];
};
constexpr HarmTab make_harm() {
    HarmTab t{};
    double a = 0.0, b = 0.0;
    for (int i = 1; i <= 64; ++i) {
        a += 1.0 / i;
        b += 1.0 / (static_cast<double>(i) * i);
        t.h1[i] = a;
        t.h2[i] = b;
    }
    return t;
}
__constant__ HarmTab kHarm = make_harm();
__device__ double harm1(int n) {
    if (n <= 64) return kHarm.h1[n];
    const double x = n;
    return log(x) + 0.57721566490153286 + 0.5 / x - 1.0 / (12.0 * x * x);
}
__device__ double harm2(int n) {
    if (n <= 64) return kHarm.h2[n];
    const double x = n + 1.0;  // pi^2 / 6 - trigamma(n + 1)
    return 1.6449340668482264 - (1.0 / x + 0.5 / (x * x) + 1.0 / (6.0 * x * x * x));
}

struct DrawSetupLds {
    double cE[kDrawPieces + 1];  // expected words before piece p (walk-major, regions high to low)
    double cV[kDrawPieces + 1];  // their variance
    int cum[kDrawWalks], hi[kDrawWalks];
    int sd[kDrawSegMax + 1];
    uint32_t blk[8][kMtN];  // the twist's LDS ring
    double shd[16];
    int shi[16];
    int nw, ktot, fail;
};

// One workgroup: the call list (kOp 0: AnchorTarget's two calls per image,
// utils/utils.py:190-202; 1: ProposalTarget's, :248-258) with the outputs that
// need no RNG, the segment plan, and the state blocks the segments read.
// The calls one chip-wide pass draws, in stream order: AnchorTarget's two per
// image (utils/utils.py:190-202), then ProposalTarget's (:248-258) -- train.py:71
// and :91 make every AnchorTarget draw before any ProposalTarget one, so both
// creators' calls can share one pass (n_at or n_pt may be 0).
struct DrawOps {
    int n_at, at_n_sample, at_pos_max;
    const int* at_npos;
    const int* at_nneg;
    int* at_sampled;
    int4* at_calls;
    int* at_jrec;
    int n_pt, pt_n_sample, pt_pos_per_image;
    const int* pt_npos;
    const int* pt_nneg;
    int4* pt_calls;
    int* pt_scount;
    int* pt_spos;
    int* pt_jrec;
};

// One workgroup: the call list with the outputs that need no RNG, the segment
// plan, and the state blocks the segments read.
__global__ __launch_bounds__(1024) void draw_setup_kernel(DrawOps ops, const uint32_t* __restrict__ rng, DrawCap cap,
                                                          float mult, int slack, DrawBufs B) {
    __shared__ DrawSetupLds L;
    const int tid = threadIdx.x;
    // ---- calls (thread = call; its jrec row is its index)
    int steps = 0, isw = 0, rec = 0;
    const int na = 2 * ops.n_at;
    if (tid < na) {
        const int n = tid >> 1, call = tid & 1;
        const int P = ops.at_npos[n], Q = ops.at_nneg[n];
        const int cnt = call ? Q : P;
        const int n_pos_max = ops.at_pos_max;
        const int pos_after = P > n_pos_max ? n_pos_max : P;
        const int m = call ? ops.at_n_sample - pos_after : n_pos_max;  // survivors
        const bool do_call = cnt > m;
        ops.at_sampled[tid] = do_call ? 1 : 0;
        ops.at_calls[tid] = do_call ? make_int4(cnt, cnt - m, cnt, 0) : make_int4(0, 0, 0, 0);
        if (do_call && cnt >= 2) {
            isw = 1;
            steps = cnt - 1;
            rec = cnt - m;
        }
    } else if (tid < na + 2 * ops.n_pt) {
        const int i = tid - na, n = i >> 1, call = i & 1;
        const int P = ops.pt_npos[n], Q = ops.pt_nneg[n];
        const int cnt = call ? Q : P;
        const int kp = P < ops.pt_pos_per_image ? P : ops.pt_pos_per_image;
        int kn = ops.pt_n_sample - kp;
        kn = Q < kn ? Q : kn;
        ops.pt_calls[i] = cnt > 0 ? make_int4(cnt, 1, call ? kn : kp, call ? kp : 0) : make_int4(0, 0, 0, 0);
        if (call == 0) {
            ops.pt_scount[n] = kp + kn;
            ops.pt_spos[n] = kp;
        }
        if (cnt >= 2) {
            isw = 1;
            steps = cnt - 1;
            rec = 1;
        }
    }
    if (tid == 0) L.fail = 0;
    int nw = 0, ktot = 0;
    const int wi = block_incl_scan(isw, L.shi, nw);
    const int ki = block_incl_scan(steps, L.shi, ktot);
    if (isw) {
        const int c = wi - 1;
        L.cum[c] = ki;
        L.hi[c] = steps;
        B.w_hi[c] = steps;
        B.w_cum[c] = ki;
        B.w_rec[c] = rec;
        B.w_row[c] = tid;
        if (steps > kDrawHiMax) L.fail = 1;
    }
    __syncthreads();
    // ---- expected words / variance per (walk, mask region), in stream order
    const int P = nw * 16;
    double e4[4], v4[4], es = 0.0, vs = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int p = tid * 4 + r;
        double E = 0.0, V = 0.0;
        if (p < P) {
            const int c = p >> 4, j = 15 - (p & 15);
            const int hic = L.hi[c], bl = 1 << j;
            if (bl <= hic) {
                const int bh = min((2 << j) - 1, hic);
                const double M = static_cast<double>(2 << j);
                E = M * (harm1(bh + 1) - harm1(bl));
                V = M * M * (harm2(bh + 1) - harm2(bl)) - E;
            }
        }
        e4[r] = E;
        v4[r] = V;
        es += E;
        vs += V;
    }
    double Etot = 0.0, Vtot = 0.0;
    double ea = block_incl_scan(es, L.shd, Etot) - es;
    double va = block_incl_scan(vs, L.shd, Vtot) - vs;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int p = tid * 4 + r;
        if (p < P) {
            L.cE[p] = ea;
            L.cV[p] = va;
        }
        ea += e4[r];
        va += v4[r];
    }
    if (tid == 0) {
        L.cE[P] = Etot;
        L.cV[P] = Vtot;
    }
    __syncthreads();
    // ---- segments: domain of the K at each segment start
    const int off0 = static_cast<int>(rng[kMtN]);
    int S = 0, SL = kSegLMax;
    if (ktot > 0) {  // short streams (ProposalTarget's) in 256-word segments: shorter lane walks
        const double span = Etot + mult * sqrt(Vtot) + slack + 64.0;
        S = static_cast<int>(ceil(span / 256.0));
        if (S <= 256) SL = 256;
        else S = static_cast<int>(ceil(span / kSegLMax));
    }
    if (S > cap.smax) {
        if (tid == 0) L.fail = 1;
        S = 0;
    }
    int D = 0, lo = 0;
    if (tid <= S && S > 0) {
        const int s = tid;
        if (s == 0) {
            lo = 0;
            D = 1;
        } else if (s == S) {
            lo = ktot;
            D = 1;
        } else {
            // the expected K at word x (the calls' mask regions, E[words per step]
            // = M / (b + 1) inverted with H(n) ~ ln(n + 1/2) + gamma) and the
            // variance of the words spent reaching it
            auto khat = [&](double x, double& var) -> double {
                if (x <= 0.0) {
                    var = 0.0;
                    return 0.0;
                }
                int a = 0, z = P;  // largest p with cE[p] <= x
                while (a < z) {
                    const int m = (a + z + 1) >> 1;
                    if (L.cE[m] <= x) a = m;
                    else z = m - 1;
                }
                if (a >= P) {
                    var = Vtot;
                    return static_cast<double>(ktot);
                }
                const int c = a >> 4, j = 15 - (a & 15);
                const int hic = L.hi[c];
                const int bl = 1 << j, bh = min((2 << j) - 1, hic);
                const double M = static_cast<double>(2 << j);
                const int K0 = L.cum[c] - hic + (hic - bh);
                double bf = (bh + 1.5) * exp(-(x - L.cE[a]) / M) - 1.5;
                bf = fmin(fmax(bf, bl - 1.0), static_cast<double>(bh));
                const double Vp = L.cV[a + 1] - L.cV[a];
                var = fmax(L.cV[a] + Vp * (bh - bf) / (bh - bl + 1.0), 0.0);
                return K0 + (bh - bf);
            };
            // the domain in WORD space: the walk's words to reach a K deviate from
            // the expectation like a Gaussian path (sigma_W), and K is read off the
            // expectation at q -+ mult sigma_W -- across mask-region edges too, where
            // the acceptance rate jumps (a linearised sigma_K under-covers there)
            const double q = static_cast<double>(s) * SL;
            double var = 0.0, vd = 0.0;
            const double kq = khat(q, var);
            const double sw = mult * sqrt(var);
            lo = max(0, static_cast<int>(floor(khat(q - sw, vd))) - slack);
            int hi = min(ktot, static_cast<int>(ceil(khat(q + sw, vd))) + slack);
            if (hi - lo + 1 > kDrawDcap) {  // narrower: only a miss more likely
                const int kc = static_cast<int>(floor(kq + 0.5));
                lo = max(0, min(kc - kDrawDcap / 2, ktot - kDrawDcap + 1));
                hi = min(ktot, lo + kDrawDcap - 1);
            }
            D = hi - lo + 1;
        }
        B.s_lo[s] = lo;
        B.s_d[s] = D;
        L.sd[s] = D;
    }
    // table offsets and wave items over segments 0 .. S-1
    const int dt = tid < S ? D : 0;
    int tabn = 0, itn = 0;
    const int ti = block_incl_scan(dt, L.shi, tabn);
    const int ii = block_incl_scan((dt + 255) >> 8, L.shi, itn);
    if (tid < S) {
        B.s_toff[tid] = ti - dt;
        B.s_item[tid] = ii - ((dt + 255) >> 8);
    }
    if (tid == 0) {
        B.s_toff[S] = tabn;
        B.s_item[S] = itn;
    }
    __syncthreads();  // L.sd
    const int ngrp = (S + kGrpG - 1) / kGrpG;
    int pg = 0, cg = 0;
    if (tid < ngrp) {
        const int gs = min(kGrpG, S - tid * kGrpG);
        pg = gs * L.sd[tid * kGrpG];
        cg = L.sd[tid * kGrpG];
    }
    int pren = 0, chn = 0;
    const int pi = block_incl_scan(pg, L.shi, pren);
    (void)block_incl_scan(cg, L.shi, chn);
    int dmx = 0;
    {
        int dm = tid < S ? D : 0;
        const int dw = static_cast<int>(__ockl_wfred_max_u32(static_cast<uint32_t>(dm)));
        if ((tid & 63) == 0) L.shi[tid >> 6] = dw;
        __syncthreads();
        for (int i = 0; i < 16; ++i) dmx = max(dmx, L.shi[i]);
        __syncthreads();
    }
    if (tid < ngrp) B.g_poff[tid] = pi - pg;
    const int nblk = S > 0 ? (off0 + S * SL - 1) / kMtN + 1 : 0;
    if (tid == 0) {
        B.g_poff[ngrp] = pren;
        if (tabn > cap.tabmax || pren > cap.premax || chn > kChainLds || nblk > cap.nbmax) L.fail = 1;
    }
    __syncthreads();
    const int fail = L.fail;
    if (tid == 0) {
        DrawHdr h;
        h.fail = fail;
        h.nw = nw;
        h.ktot = ktot;
        h.nseg = fail ? 0 : S;
        h.ngrp = fail ? 0 : ngrp;
        h.nblk = nblk;
        h.off0 = off0;
        h.dmax = dmx;
        h.miss = -1;
        h.seg_l = SL;
        *B.hdr = h;
    }
    if (fail || nblk == 0) return;  // (block-uniform)
    // ---- the state blocks the segments read: block 0 is the key handed in.
    // Waves 0-3 twist block b from block b - 1 in an LDS ring of kTwRing blocks
    // (read, mix, write: the only work between two barriers); waves 4-15 copy
    // block b - 1 out (raw, and tempered from the draws' first word on) meanwhile.
    constexpr int kTwRing = 8;
    for (int i = tid; i < kMtN; i += 1024) L.blk[0][i] = rng[i];
    __syncthreads();
    for (int b = 1; b <= nblk; ++b) {
        if (tid < 256) {
            const int t = tid;
            if (b < nblk && t < kMtN - kMtM) {  // as mt_twist: words t, t + 227, t + 454
                const uint32_t* old = L.blk[(b - 1) % kTwRing];
                uint32_t* nw_ = L.blk[b % kTwRing];
                // every LDS read first (clamped indices): one round trip per block
                const uint32_t o0 = old[t], o1 = old[t + 1], o397 = old[t + kMtM];
                const uint32_t o227 = old[t + 227], o228 = old[t + 228];
                const uint32_t o454 = old[min(t + 454, kMtN - 1)], o455 = old[min(t + 455, kMtN - 1)];
                const uint32_t z0 = old[0], z1 = old[1], z397 = old[kMtM];
                const uint32_t a = o397 ^ mt_mix(o0, o1);
                const uint32_t bb = a ^ mt_mix(o227, o228);
                nw_[t] = a;
                nw_[t + 227] = bb;
                if (t + 454 <= kMtN - 1) {
                    // word 623 wraps to the new word 0 (recomputed here)
                    const uint32_t hi_in = t + 454 < kMtN - 1 ? o455 : (z397 ^ mt_mix(z0, z1));
                    nw_[t + 454] = bb ^ mt_mix(o454, hi_in);
                }
            }
        } else {  // copy block b - 1 out
            const uint32_t* src = L.blk[(b - 1) % kTwRing];
            uint32_t* rg = B.raw + static_cast<size_t>(b - 1) * kMtN;
            const int a0 = (b - 1) * kMtN - off0;  // tw index of the block's word 0
            for (int i = tid - 256; i < kMtN; i += 768) {
                const uint32_t v = src[i];
                rg[i] = v;
                if (a0 + i >= 0) B.tw[a0 + i] = mt_temper(v);
            }
        }
        // LDS-only barrier: the copies' global stores need not land before the next
        // twist (__syncthreads would wait for them)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

// One workgroup per 256 entering K's of a segment (a wave per 64): the
// segment's words staged in LDS, each lane walks them from its own K.  Per
// word: v = w & mask, accept iff v < bound + 1, bound -= accepted (3 VALU, the
// word a broadcast LDS read per four); the masks and the walks' ends are
// refreshed only after `rem` words, the wave's least distance (in acceptances)
// to a lane's region edge or walk end.
__global__ __launch_bounds__(256) void draw_table_kernel(const DrawHdr* __restrict__ hdr, DrawBufs B) {
    __shared__ int cum[kDrawWalks + 1];
    __shared__ int his[kDrawWalks + 1];
    __shared__ int item[kDrawSegMax + 1];
    __shared__ uint4 words[kSegLMax / 4];
    if (hdr->fail) return;
    const int nw = hdr->nw, ktot = hdr->ktot, S = hdr->nseg, L = hdr->seg_l;
    for (int i = threadIdx.x; i < nw; i += 256) {
        cum[i] = B.w_cum[i];
        his[i] = B.w_hi[i];
    }
    for (int i = threadIdx.x; i <= S; i += 256) item[i] = B.s_item[i];
    if (threadIdx.x == 0) {
        cum[nw] = 0x7fffffff;
        his[nw] = 0;
    }
    __syncthreads();
    const int nitems = item[S];
    const int lane = threadIdx.x & 63;
    for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
        int a = 0, z = S - 1;  // segment: largest s with item[s] <= it
        while (a < z) {
            const int m = (a + z + 1) >> 1;
            if (item[m] <= it) a = m;
            else z = m - 1;
        }
        const int s = __builtin_amdgcn_readfirstlane(a);
        {
            const uint4* src = reinterpret_cast<const uint4*>(B.tw + static_cast<size_t>(s) * L);
            for (int i = threadIdx.x; i < L / 4; i += 256) words[i] = src[i];
        }
        __syncthreads();
        const int k = (it - item[s]) * 256 + static_cast<int>(threadIdx.x);
        const int D = B.s_d[s];
        if (__builtin_amdgcn_readfirstlane(k - lane) < D) {  // (a wave past the domain skips)
            const int Dn = B.s_d[s + 1];
            const int lon = B.s_lo[s + 1];
            const int K = B.s_lo[s] + k;
            int c = 0;
            {
                int l = 0, r = nw;  // first walk with cum > K (nw: the draws are over)
                while (l < r) {
                    const int m = (l + r) >> 1;
                    if (cum[m] > K) r = m;
                    else l = m + 1;
                }
                c = l;
            }
            uint32_t bnd = c < nw ? static_cast<uint32_t>(cum[c] - K) + 1u : 0u;  // bound + 1; 0: done
            uint32_t msk = 0;
            int rem = 0;
            uint4 wn[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) wn[u] = words[u];
            for (int t0 = 0; t0 < L; t0 += 16) {
                uint32_t w[16];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    w[4 * u] = wn[u].x;
                    w[4 * u + 1] = wn[u].y;
                    w[4 * u + 2] = wn[u].z;
                    w[4 * u + 3] = wn[u].w;
                }
                const int tn = t0 + 16 < L ? t0 + 16 : t0;
#pragma unroll
                for (int u = 0; u < 4; ++u) wn[u] = words[tn / 4 + u];
                if (rem >= 16) {  // no lane reaches a region edge or walk end
                    // accepted iff (w & mask) < bound + 1, both < 2^17: the sign of their
                    // difference, all in VGPRs (a compare would route every word's decision
                    // through VCC, an SGPR round trip per word on the dependency chain)
#pragma unroll
                    for (int u = 0; u < 16; ++u) bnd -= ((w[u] & msk) - bnd) >> 31;
                    rem -= 16;
                } else {
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        if (rem == 0) {
                            if (bnd == 1u) {  // walk c ended: the next call's first bound
                                ++c;
                                bnd = c < nw ? static_cast<uint32_t>(his[c]) + 1u : 0u;
                            }
                            const uint32_t b = bnd - 1u;
                            msk = 0xffffffffu >> __builtin_clz(b | 1u);
                            const uint32_t run = bnd ? b - (msk >> 1) : 0x7fffffffu;  // >= 1
                            rem = static_cast<int>(__ockl_wfred_min_u32(run));
                        }
                        bnd -= ((w[u] & msk) - bnd) >> 31;
                        --rem;
                    }
                }
            }
            if (k < D) {
                const int Ko = c < nw ? cum[c] - static_cast<int>(bnd - 1u) : ktot;
                const int rel = Ko - lon;
                B.tab[B.s_toff[s] + k] = (rel >= 0 && rel < Dn) ? static_cast<uint16_t>(rel) : kMiss;
            }
        }
        __syncthreads();  // the words are restaged next item
    }
}

// One workgroup per group of kGrpG segments: its tables staged in LDS, each
// entering K of the group's first segment followed through them; the K after
// every segment is kept (pre), the last one is the group's composite.
__global__ __launch_bounds__(1024) void draw_group_kernel(const DrawHdr* __restrict__ hdr, DrawBufs B) {
    __shared__ uint16_t st[kGrpG * kDrawDcap];
    __shared__ int soff[kGrpG + 1];
    if (hdr->fail) return;
    const int g = blockIdx.x;
    const int S = hdr->nseg;
    if (g >= hdr->ngrp) return;
    const int s0 = g * kGrpG, gs = min(kGrpG, S - s0);
    if (threadIdx.x <= gs) soff[threadIdx.x] = B.s_toff[s0 + threadIdx.x];
    __syncthreads();
    const int base = soff[0], n = soff[gs] - base;
    for (int i = threadIdx.x; i < n; i += 1024) st[i] = B.tab[base + i];
    __syncthreads();
    const int D0 = B.s_d[s0];
    uint16_t* pg = B.pre + B.g_poff[g];
    for (int k = threadIdx.x; k < D0; k += 1024) {
        uint32_t v = static_cast<uint32_t>(k);
        for (int j = 0; j < gs; ++j) {
            if (v != kMiss) v = st[soff[j] - base + v];
            pg[static_cast<size_t>(j) * D0 + k] = static_cast<uint16_t>(v);
        }
    }
}

// One workgroup: the group composites staged in LDS and chained from K = 0
// (one lane), then the exact K at every segment start from the groups'
// prefix tables.  A miss anywhere on the path hands the draws to the serial
// sampler (hdr.fail = 2).
__global__ __launch_bounds__(1024) void draw_chain_kernel(DrawHdr* __restrict__ hdr, DrawBufs B) {
    __shared__ uint16_t comp[kChainLds];
    __shared__ int coff[kDrawSegMax / kGrpG + 2];
    __shared__ int d0[kDrawSegMax / kGrpG + 2];
    __shared__ int vg[kDrawSegMax / kGrpG + 2];
    __shared__ int bad;
    if (hdr->fail) return;
    const int S = hdr->nseg, ngrp = hdr->ngrp;
    if (S == 0) return;
    const int tid = threadIdx.x;
    if (tid < ngrp) d0[tid] = B.s_d[tid * kGrpG];
    if (tid == 0) bad = 0;
    __syncthreads();
    if (tid == 0) {
        int o = 0;
        for (int g = 0; g < ngrp; ++g) {
            coff[g] = o;
            o += d0[g];
        }
        coff[ngrp] = o;
    }
    __syncthreads();
    // every composite entry loaded at once (one memory latency, not one per group)
    const int ntot = coff[ngrp];
    for (int i = tid; i < ntot; i += 1024) {
        int a = 0, z = ngrp - 1;  // group: largest g with coff[g] <= i
        while (a < z) {
            const int m = (a + z + 1) >> 1;
            if (coff[m] <= i) a = m;
            else z = m - 1;
        }
        const int gs = min(kGrpG, S - a * kGrpG);
        comp[i] = B.pre[B.g_poff[a] + static_cast<size_t>(gs - 1) * d0[a] + (i - coff[a])];
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t v = 0;  // K = 0 at the stream start: entry 0 of segment 0's domain {0}
        for (int g = 0; g < ngrp; ++g) {
            vg[g] = static_cast<int>(v);
            v = comp[coff[g] + v];
            if (v == kMiss) {
                bad = 1 + g;
                break;
            }
        }
    }
    __syncthreads();
    if (bad) {
        if (tid == 0) {
            hdr->fail = 2;
            hdr->miss = bad - 1;
        }
        return;
    }
    for (int s = tid; s <= S; s += 1024) {
        int K = 0;
        if (s > 0) {
            const int g = (s - 1) / kGrpG, j = (s - 1) % kGrpG;
            K = B.s_lo[s] + B.pre[B.g_poff[g] + static_cast<size_t>(j) * d0[g] + vg[g]];
        }
        B.kseg[s] = K;
    }
}

// One wave per segment: the segment's words walked exactly from the K the
// chain found, 64 at a time (ballot fixed point, as the serial walk's), when
// the segment holds a recorded swap or the stream's last draw; the last draw's
// segment hands the state back (numpy's pos = 1..624 within the key block).
__global__ __launch_bounds__(64) void draw_record_kernel(const DrawHdr* __restrict__ hdr, DrawBufs B,
                                                         DrawOps ops, uint32_t* __restrict__ rng) {
    __shared__ int cum[kDrawWalks + 1];
    __shared__ int rec[kDrawWalks];
    __shared__ int row[kDrawWalks];
    if (hdr->fail) return;
    const int s = blockIdx.x;
    const int S = hdr->nseg;
    if (s >= S) return;
    const int nw = hdr->nw, ktot = hdr->ktot, off0 = hdr->off0;
    const int lane = threadIdx.x;
    const int K0 = B.kseg[s], K1 = B.kseg[s + 1];
    if (K0 == K1) return;  // no acceptance in this segment
    for (int i = lane; i < nw; i += 64) {
        cum[i] = B.w_cum[i];
        rec[i] = B.w_rec[i];
        row[i] = B.w_row[i];
    }
    if (lane == 0) cum[nw] = 0x7fffffff;
    __syncthreads();
    bool want = K1 == ktot;  // the stream's last acceptance is in here
    for (int c = lane; c < nw; c += 64) {
        const int hic = c ? cum[c] - cum[c - 1] : cum[0];
        const int st = cum[c] - hic;  // K at the walk's first step (bound hic)
        const int r1 = st + hic - rec[c];  // K at its lowest recorded bound
        if (rec[c] <= hic && st < K1 && r1 >= K0) want = true;
    }
    if (!__builtin_amdgcn_ballot_w64(want)) return;
    auto walk_of = [&](int K) {
        int l = 0, r = nw;
        while (l < r) {
            const int m = (l + r) >> 1;
            if (cum[m] > K) r = m;
            else l = m + 1;
        }
        return l;
    };
    const int L = hdr->seg_l;
    int cw = walk_of(K0);  // the walk of the chunk's first K, carried across chunks
    const uint32_t* wp = B.tw + static_cast<size_t>(s) * L;
    uint32_t wv[kSegLMax / 64];  // every chunk's word loaded at once (one memory latency)
#pragma unroll
    for (int ch = 0; ch < kSegLMax / 64; ++ch) wv[ch] = ch * 64 < L ? wp[ch * 64 + lane] : 0u;
    int Kc = K0, qend = -1;
#pragma unroll
    for (int ch = 0; ch < kSegLMax / 64; ++ch) {
        if (ch * 64 >= L || Kc >= K1) break;
        const uint32_t w = wv[ch];
        while (cw < nw && cum[cw] <= Kc) ++cw;
        const int c0 = cw;
        const bool one = c0 < nw && Kc + 64 <= cum[c0];  // the chunk stays in walk c0
        const uint32_t b0 = c0 < nw ? static_cast<uint32_t>(cum[c0] - Kc) : 0u;
        const float pa = (static_cast<float>(b0) + 1.0f) / (static_cast<float>(mask_for(b0 | 1u)) + 1.0f);
        uint64_t ac = 0;
        int c = c0, K = Kc;
        uint32_t b = 0;
        bool acc = false;
        int below = static_cast<int>(static_cast<float>(lane) * pa);
        for (int itn = 0;; ++itn) {
            K = Kc + below;
            c = c0;  // the lane's walk: c0 or a few past it (the chunk accepts <= 64)
            if (!one)
                while (c < nw && cum[c] <= K) ++c;
            b = (c < nw && K < ktot) ? static_cast<uint32_t>(cum[c] - K) : 0u;
            acc = max(w & mask_nz(b), 1u) <= b;
            const uint64_t nac = __builtin_amdgcn_ballot_w64(acc);
            if (itn > 0 && nac == ac) break;
            ac = nac;
            below = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(ac >> 32),
                                                                __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(ac), 0u)));
        }
        if (acc) {
            if (static_cast<int>(b) >= rec[c]) {
                const int r = row[c], na = 2 * ops.n_at;
                int* jrow = r < na ? ops.at_jrec + static_cast<size_t>(r) * kMaxKeep
                                   : ops.pt_jrec + static_cast<size_t>(r - na) * kMaxKeep;
                jrow[static_cast<int>(b) - rec[c]] = static_cast<int>(w & mask_nz(b));
            }
            if (K + 1 == ktot) qend = s * L + ch * 64 + lane + 1;
        }
        Kc += __popcll(ac);
    }
    const int qe = static_cast<int>(__ockl_wfred_max_i32(qend));
    if (qe > 0) {
        const int A = off0 + qe;  // words [off0, A) consumed: the key is block (A-1)/624
        const int blk = (A - 1) / kMtN;
        const uint32_t* src = B.raw + static_cast<size_t>(blk) * kMtN;
        for (int i = lane; i < kMtN; i += 64) rng[i] = src[i];
        if (lane == 0) rng[kMtN] = static_cast<uint32_t>((A - 1) % kMtN + 1);
    }
}

// "chip_only" (tests): when the plan failed nothing was drawn, so the finishing
// kernels get no calls and no samples rather than stale swap records.
__global__ __launch_bounds__(256) void draw_poison_kernel(const DrawHdr* __restrict__ hdr, DrawOps ops) {
    if (hdr->fail == 0) return;
    for (int i = threadIdx.x; i < 2 * ops.n_at; i += blockDim.x) {
        ops.at_calls[i] = make_int4(0, 0, 0, 0);
        ops.at_sampled[i] = 0;
    }
    for (int i = threadIdx.x; i < 2 * ops.n_pt; i += blockDim.x) {
        ops.pt_calls[i] = make_int4(0, 0, 0, 0);
        if ((i & 1) == 0) {
            ops.pt_scount[i >> 1] = 0;
            ops.pt_spos[i >> 1] = 0;
        }
    }
}

// grid N x n_sample: sample_roi, normalised gt_roi_reg and gt_roi_label
// (utils/utils.py:265-276).  Rows past the sample count are zero.
struct RegNorm {
    double mean[4];
    double stdv[4];
};

__global__ __launch_bounds__(128) void pt_finish_kernel(
    int stride, int n_sample, const double* __restrict__ roi_all, const int32_t* __restrict__ assign,
    const double* __restrict__ gt, const double* __restrict__ gl, const int* __restrict__ gcount,
    int Gp, const int* __restrict__ sample, const int* __restrict__ scount,
    const int* __restrict__ spos, RegNorm nrm, double* __restrict__ s_roi, double* __restrict__ s_reg,
    double* __restrict__ s_lab) {
    const int n = blockIdx.x;
    const int s = threadIdx.x + blockIdx.y * 128;
    if (s >= n_sample) return;
    const size_t o = static_cast<size_t>(n) * n_sample + s;
    if (s >= scount[n]) {
        for (int c = 0; c < 4; ++c) s_roi[o * 4 + c] = s_reg[o * 4 + c] = 0.0;
        s_lab[o] = 0.0;
        return;
    }
    const int t = sample[o];
    const double* r = roi_all + (static_cast<size_t>(n) * stride + t) * 4;
    for (int c = 0; c < 4; ++c) s_roi[o * 4 + c] = r[c];
    const int G = gcount[n];
    if (G == 0) {
        for (int c = 0; c < 4; ++c) s_reg[o * 4 + c] = 0.0;
        s_lab[o] = 0.0;
        return;
    }
    const int g = assign[static_cast<size_t>(n) * stride + t];
    const double* b = gt + (static_cast<size_t>(n) * Gp + g) * 4;
    const double ah = r[2] - r[0], aw = r[3] - r[1];
    const double acx = (r[2] + r[0]) / 2.0, acy = (r[1] + r[3]) / 2.0;
    const double bh = b[2] - b[0], bw = b[3] - b[1];
    const double bcx = (b[2] + b[0]) / 2.0, bcy = (b[1] + b[3]) / 2.0;
    double v[4];
    v[0] = (bcx - acx) / ah;
    v[1] = (bcy - acy) / aw;
    v[2] = log(bh / ah);
    v[3] = log(bw / aw);
    for (int c = 0; c < 4; ++c) s_reg[o * 4 + c] = (v[c] - nrm.mean[c]) / nrm.stdv[c];
    s_lab[o] = s < spos[n] ? gl[static_cast<size_t>(n) * Gp + g] : 0.0;
}

// ------------------------------------------------------ generic bbox_iou op
template <class TA, class TB, class TO>
__global__ __launch_bounds__(256) void bbox_iou_kernel(const TA* __restrict__ a, int64_t na,
                                                       const TB* __restrict__ b, int64_t nb,
                                                       TO* __restrict__ out) {
    const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (idx >= na * nb) return;
    const int64_t i = idx / nb, j = idx - i * nb;
    const TA* p = a + i * 4;
    const TB* q = b + j * 4;
    if (sizeof(TO) == 4) {  // both fp32: numpy computes in fp32
        float tl0 = np_max<float>(p[0], q[0]), tl1 = np_max<float>(p[1], q[1]);
        float br0 = np_min<float>(p[2], q[2]), br1 = np_min<float>(p[3], q[3]);
        float inter = (br0 - tl0) * (br1 - tl1);
        inter = inter * ((tl0 < br0 && tl1 < br1) ? 1.0f : 0.0f);
        float aa = area_np(reinterpret_cast<const float*>(p));
        float ab = area_np(reinterpret_cast<const float*>(q));
        float uni = aa + ab;
        uni = uni - inter;
        out[idx] = static_cast<TO>(inter / uni);
    } else {
        const double qa[4] = {static_cast<double>(q[0]), static_cast<double>(q[1]),
                              static_cast<double>(q[2]), static_cast<double>(q[3])};
        const double ab = static_cast<double>(area_np(q));
        out[idx] = static_cast<TO>(iou_np(p, static_cast<double>(area_np(p)), qa, ab));
    }
}

// utils/utils.py:75-100 with numpy promotion: anchor statistics in the
// anchors' dtype, box statistics in the boxes' dtype, result fp64.
template <class TA, class TB>
__global__ __launch_bounds__(256) void bbox2reg_kernel(const TA* __restrict__ a,
                                                       const TB* __restrict__ b, int64_t n,
                                                       double* __restrict__ out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const TA* p = a + i * 4;
    const TB* q = b + i * 4;
    const TA ah = p[2] - p[0], aw = p[3] - p[1];
    const TA acx = (p[2] + p[0]) / TA(2), acy = (p[1] + p[3]) / TA(2);
    const TB bh = q[2] - q[0], bw = q[3] - q[1];
    const TB bcx = (q[2] + q[0]) / TB(2), bcy = (q[1] + q[3]) / TB(2);
    double* o = out + i * 4;
    if (sizeof(TA) == 4 && sizeof(TB) == 4) {  // both fp32: numpy computes in fp32, stores fp64
        o[0] = static_cast<double>((bcx - acx) / ah);
        o[1] = static_cast<double>((bcy - acy) / aw);
        o[2] = static_cast<double>(logf(static_cast<float>(bh / ah)));
        o[3] = static_cast<double>(logf(static_cast<float>(bw / aw)));
    } else {
        o[0] = (static_cast<double>(bcx) - static_cast<double>(acx)) / static_cast<double>(ah);
        o[1] = (static_cast<double>(bcy) - static_cast<double>(acy)) / static_cast<double>(aw);
        o[2] = log(static_cast<double>(bh) / static_cast<double>(ah));
        o[3] = log(static_cast<double>(bw) / static_cast<double>(aw));
    }
}

}  // namespace frcnn

using namespace frcnn;

// =========================================================== C-ABI wrappers
namespace {
struct AtWs {
    double* gt;
    double* gl;
    int* gcount;
    int32_t* row_arg;
    double* row_max;
    double* col_v;
    int* col_i;
    int8_t* label0;
    int* pos_list;
    int* neg_list;
    int* npos;
    int* nneg;
    uint8_t* keep;
    int* sampled;
    int4* calls;  // [2N] per choice() call: cnt (0: none), lowest recorded step, p_hi, offset
    int* jrec;    // [2N][kMaxKeep] recorded swaps
    DrawCap cap;  // the chip-wide draws' capacity (cap.smax == 0: the walk only)
    DrawBufs draw;
    size_t bytes;
};

// Capacity of the chip-wide draws for a stream of at most steps_cap Fisher-Yates
// steps (each takes < 2 words on average): past it the plan fails and the walk runs.
DrawCap draw_cap(int N, int64_t steps_cap) {
    DrawCap c{};
    if (N <= 0 || 2 * N > kDrawWalks || steps_cap <= 0) return c;
    const double words = 2.0 * static_cast<double>(steps_cap) + 64.0 * std::sqrt(static_cast<double>(steps_cap)) + 4096.0;
    // 1024-word segments, or 256-word ones when a stream fits 256 of them
    const double s1024 = words / kSegLMax + 2.0, s256 = std::min(words / 256.0 + 2.0, 258.0);
    c.smax = static_cast<int>(std::min(std::max(s1024, s256), static_cast<double>(kDrawSegMax - 1)));
    c.nbmax = (kMtN + static_cast<int>(std::min(words + 4.0 * kSegLMax, 1.1e6))) / kMtN + 2;
    c.tabmax = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(c.smax) * kDrawDcap, int64_t{1} << 22));
    c.premax = c.tabmax;
    return c;
}
DrawBufs carve_draw(Carver& c, const DrawCap& cap) {
    DrawBufs b{};
    if (cap.smax == 0) return b;
    b.hdr = c.take<DrawHdr>(1);
    b.w_hi = c.take<int>(kDrawWalks);
    b.w_cum = c.take<int>(kDrawWalks);
    b.w_rec = c.take<int>(kDrawWalks);
    b.w_row = c.take<int>(kDrawWalks);
    b.s_lo = c.take<int>(cap.smax + 1);
    b.s_d = c.take<int>(cap.smax + 1);
    b.s_toff = c.take<int>(cap.smax + 1);
    b.s_item = c.take<int>(cap.smax + 1);
    b.g_poff = c.take<int>(cap.smax / kGrpG + 2);
    b.kseg = c.take<int>(cap.smax + 1);
    b.tab = c.take<uint16_t>(cap.tabmax);
    b.pre = c.take<uint16_t>(cap.premax);
    b.raw = c.take<uint32_t>(static_cast<size_t>(cap.nbmax) * kMtN);
    b.tw = c.take<uint32_t>(static_cast<size_t>(cap.nbmax) * kMtN);
    return b;
}

// The serial samplers' arguments (the walk: the fallback, and the path for
// workspaces without a chip-wide part).
struct SerialAt {
    int N, A, n_sample, n_pos_max;
    const int* pos_list;
    const int* neg_list;
    const int* npos;
    const int* nneg;
    int* sampled;
    int4* calls;
    int* jrec;
};
struct SerialPt {
    int N, stride, n_sample, pos_per_image;
    const int* pos_list;
    const int* neg_list;
    const int* npos;
    const int* nneg;
    int* scount;
    int* spos;
    int4* calls;
    int* jrec;
};

// The draws of ops on the stream rng: chip-wide (setup, segment tables, group
// composites, chain, exact walks of the recorded segments) with the serial
// samplers behind, gated on the plan's fail flag; the serial samplers alone on
// the "walk" path or without a chip-wide workspace part.
int launch_draws(const DrawOps& ops, const SerialAt* at, const SerialPt* pt, uint32_t* rng, const DrawCap& cap,
                 const DrawBufs& B, hipStream_t st) {
    const int path = path_cfg().sampler;
    const bool chip = path != kPathWalk && cap.smax > 0 && 2 * (ops.n_at + ops.n_pt) <= kDrawWalks;
    if (chip) {
#ifndef FRCNN_DRAW_SIGMAS
#define FRCNN_DRAW_SIGMAS 4.0f  // domain half-width in sigma_W (worst of 140 simulated cfg5 paths: 3.7)
#endif
        const float mult = path == kPathChipTight ? 0.0f : FRCNN_DRAW_SIGMAS;
        const int slack = path == kPathChipTight ? 0 : 16;
        hipLaunchKernelGGL(draw_setup_kernel, dim3(1), dim3(1024), 0, st, ops, rng, cap, mult, slack, B);
        FRCNN_LAUNCH_CHECK("draw_setup_kernel");
#ifndef FRCNN_TABLE_WGS
#define FRCNN_TABLE_WGS 2048  // 8 waves per SIMD
#endif
        hipLaunchKernelGGL(draw_table_kernel, dim3(FRCNN_TABLE_WGS), dim3(256), 0, st, B.hdr, B);
        FRCNN_LAUNCH_CHECK("draw_table_kernel");
        hipLaunchKernelGGL(draw_group_kernel, dim3((cap.smax + kGrpG - 1) / kGrpG), dim3(1024), 0, st, B.hdr, B);
        FRCNN_LAUNCH_CHECK("draw_group_kernel");
        hipLaunchKernelGGL(draw_chain_kernel, dim3(1), dim3(1024), 0, st, B.hdr, B);
        FRCNN_LAUNCH_CHECK("draw_chain_kernel");
        hipLaunchKernelGGL(draw_record_kernel, dim3(cap.smax), dim3(64), 0, st, B.hdr, B, ops, rng);
        FRCNN_LAUNCH_CHECK("draw_record_kernel");
        if (path == kPathChipOnly) {  // (tests) no walk behind: a failed plan leaves no calls
            hipLaunchKernelGGL(draw_poison_kernel, dim3(1), dim3(256), 0, st, B.hdr, ops);
            FRCNN_LAUNCH_CHECK("draw_poison_kernel");
            return FRCNN_OK;
        }
    }
    const int* gate = chip ? reinterpret_cast<const int*>(B.hdr) : nullptr;
    if (at && pt) {
        hipLaunchKernelGGL(target_sample_kernel, dim3(1), dim3(kSampThreads), 0, st, at->N, at->n_sample,
                           at->n_pos_max, at->npos, at->nneg, at->sampled, at->calls, at->jrec, pt->N, pt->n_sample,
                           pt->pos_per_image, pt->npos, pt->nneg, pt->scount, pt->spos, pt->calls, pt->jrec, rng,
                           gate);
        FRCNN_LAUNCH_CHECK("target_sample_kernel");
        return FRCNN_OK;
    }
    if (at) {
        hipLaunchKernelGGL(at_sample_kernel, dim3(1), dim3(kSampThreads), 0, st, at->N, at->A, at->n_sample,
                           at->n_pos_max, at->pos_list, at->neg_list, at->npos, at->nneg, rng, at->sampled, at->calls,
                           at->jrec, gate);
        FRCNN_LAUNCH_CHECK("at_sample_kernel");
    }
    if (pt) {
        hipLaunchKernelGGL(pt_sample_kernel, dim3(1), dim3(kSampThreads), 0, st, pt->N, pt->stride, pt->n_sample,
                           pt->pos_per_image, pt->pos_list, pt->neg_list, pt->npos, pt->nneg, rng, pt->scount,
                           pt->spos, pt->calls, pt->jrec, gate);
        FRCNN_LAUNCH_CHECK("pt_sample_kernel");
    }
    return FRCNN_OK;
}

AtWs carve_at(void* ws, int N, int A, int Gp) {
    Carver c(ws);
    AtWs w{};
    const int nblk = (A + 255) / 256;
    w.gt = c.take<double>(static_cast<size_t>(N) * Gp * 4);
    w.gl = c.take<double>(static_cast<size_t>(N) * Gp);
    w.gcount = c.take<int>(N);
    w.row_arg = c.take<int32_t>(static_cast<size_t>(N) * A);
    w.row_max = c.take<double>(static_cast<size_t>(N) * A);
    w.col_v = c.take<double>(static_cast<size_t>(N) * nblk * Gp);
    w.col_i = c.take<int>(static_cast<size_t>(N) * nblk * Gp);
    w.label0 = c.take<int8_t>(static_cast<size_t>(N) * A);
    w.pos_list = c.take<int>(static_cast<size_t>(N) * A);
    w.neg_list = c.take<int>(static_cast<size_t>(N) * A);
    w.npos = c.take<int>(N);
    w.nneg = c.take<int>(N);
    w.keep = c.take<uint8_t>(static_cast<size_t>(N) * A);
    w.sampled = c.take<int>(2 * N);
    w.calls = c.take<int4>(2 * N);
    w.jrec = c.take<int>(static_cast<size_t>(2 * N) * kMaxKeep);
    w.cap = draw_cap(N, static_cast<int64_t>(N) * A);
    w.draw = carve_draw(c, w.cap);
    w.bytes = c.used();
    return w;
}

void at_ops(const AtWs& w, int N, int A, int n_sample, int n_pos_max, DrawOps& ops, SerialAt& at) {
    ops.n_at = N;
    ops.at_n_sample = n_sample;
    ops.at_pos_max = n_pos_max;
    ops.at_npos = w.npos;
    ops.at_nneg = w.nneg;
    ops.at_sampled = w.sampled;
    ops.at_calls = w.calls;
    ops.at_jrec = w.jrec;
    at = SerialAt{N, A, n_sample, n_pos_max, w.pos_list, w.neg_list, w.npos, w.nneg, w.sampled, w.calls, w.jrec};
}


}  // namespace

#ifdef FRCNN_SAMPLER_PROF
extern "C" int frcnn_debug_sampler_prof(unsigned long long* out, int reset) {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_samp_prof), sizeof(unsigned long long) * 16);
    if (reset) {
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_samp_prof), z, sizeof(z));
    }
    return 0;
}
#endif

extern "C" size_t frcnn_anchor_target_workspace_size(int N, int A, int G) {
    if (N <= 0 || A <= 0 || G < 0) return 0;
    return carve_at(nullptr, N, A, G > 0 ? G : 1).bytes;
}

extern "C" int frcnn_anchor_target_prepare(int N, int A, int G, const float* anchors, const double* boxes,
                                           const double* labels, double pos_iou_thresh,
                                           double neg_iou_thresh, void* workspace, size_t ws_bytes,
                                           void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && A > 0 && G >= 0 && G <= kMaxG,
                  "frcnn_anchor_target_prepare: need 0 < N <= 65535, A > 0, 0 <= G <= %d", kMaxG);
    FRCNN_REQUIRE(anchors, "frcnn_anchor_target_prepare: null anchors");
    FRCNN_REQUIRE(G == 0 || (boxes && labels), "frcnn_anchor_target_prepare: null boxes");
    const int Gp = G > 0 ? G : 1;
    AtWs w = carve_at(workspace, N, A, Gp);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_anchor_target_prepare: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    hipStream_t st = as_stream(stream);
    if (G > 0) {
        hipLaunchKernelGGL(gt_compact_kernel, dim3(N), dim3(64), 0, st, boxes, labels, G, w.gt, w.gl,
                           w.gcount);
        FRCNN_LAUNCH_CHECK("gt_compact_kernel");
    } else if (hipMemsetAsync(w.gcount, 0, sizeof(int) * N, st) != hipSuccess) {
        return check_launch("frcnn_anchor_target_prepare memset");
    }
    const int nblk = (A + 255) / 256;
    hipLaunchKernelGGL(at_iou_kernel, dim3(nblk, N), dim3(256), 0, st, anchors, A, w.gt, w.gcount,
                       Gp, w.row_arg, w.row_max, w.col_v, w.col_i);
    FRCNN_LAUNCH_CHECK("at_iou_kernel");
    hipLaunchKernelGGL(at_label_kernel, dim3(N), dim3(1024), 0, st, A, Gp, nblk, w.gcount,
                       w.row_max, w.col_v, w.col_i, neg_iou_thresh, pos_iou_thresh, w.row_arg,
                       w.label0, w.pos_list, w.neg_list, w.npos, w.nneg);
    FRCNN_LAUNCH_CHECK("at_label_kernel");
    if (hipMemsetAsync(w.keep, 0, static_cast<size_t>(N) * A, st) != hipSuccess)
        return check_launch("frcnn_anchor_target_prepare memset");
    return FRCNN_OK;
}

extern "C" int frcnn_anchor_target_draw(int N, int A, int G, int n_sample, double pos_ratio, uint32_t* rng_state,
                                        void* workspace, size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && A > 0 && G >= 0 && G <= kMaxG,
                  "frcnn_anchor_target_draw: need 0 < N <= 65535, A > 0, 0 <= G <= %d", kMaxG);
    const int n_pos_max = static_cast<int>(pos_ratio * n_sample);  // int(0.5*256) (utils/utils.py:190)
    FRCNN_REQUIRE(n_sample > 0 && n_sample - (n_pos_max < 0 ? 0 : n_pos_max) <= kMaxKeep && n_pos_max <= kMaxKeep,
                  "frcnn_anchor_target_draw: n_sample must be in 1..%d per choice() call", kMaxKeep);
    const int Gp = G > 0 ? G : 1;
    AtWs w = carve_at(workspace, N, A, Gp);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_anchor_target_draw: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    hipStream_t st = as_stream(stream);
    if (rng_state) {
        DrawOps ops{};
        SerialAt at{};
        at_ops(w, N, A, n_sample, n_pos_max, ops, at);
        const int rc = launch_draws(ops, &at, nullptr, rng_state, w.cap, w.draw, st);
        if (rc != FRCNN_OK) return rc;
    } else if (hipMemsetAsync(w.sampled, 0, sizeof(int) * 2 * N, st) != hipSuccess ||
               hipMemsetAsync(w.calls, 0, sizeof(int4) * 2 * N, st) != hipSuccess) {
        return check_launch("frcnn_anchor_target_draw memset");
    }
    return FRCNN_OK;
}

// The chip-wide draws' plan header of the last frcnn_anchor_target_draw on this
// workspace (synchronous): out[9] = fail, walks, steps, segments, groups, state
// blocks, start pos, widest domain, missed group; rc 1 when the workspace has no
// chip-wide part (the walk only).
static int draw_status(const DrawBufs& d, const DrawCap& cap, int* out) {
    if (cap.smax == 0) return 1;
    DrawHdr h{};
    if (hipMemcpy(&h, d.hdr, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return check_launch("draw_status copy");
    const int v[9] = {h.fail, h.nw, h.ktot, h.nseg, h.ngrp, h.nblk, h.off0, h.dmax, h.miss};
    for (int i = 0; i < 9; ++i) out[i] = v[i];
    return FRCNN_OK;
}

extern "C" int frcnn_anchor_target_draw_status(int N, int A, int G, const void* workspace, size_t ws_bytes,
                                               int* out) {
    FRCNN_REQUIRE(N > 0 && A > 0 && G >= 0 && out, "frcnn_anchor_target_draw_status: bad argument");
    AtWs w = carve_at(const_cast<void*>(workspace), N, A, G > 0 ? G : 1);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_anchor_target_draw_status: workspace too small");
    return draw_status(w.draw, w.cap, out);
}

extern "C" int frcnn_anchor_target_finish(int N, int A, int G, const float* anchors, double* reg, int32_t* label,
                                          int32_t* argmax, double* max_iou, void* workspace, size_t ws_bytes,
                                          void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && A > 0 && G >= 0 && G <= kMaxG,
                  "frcnn_anchor_target_finish: need 0 < N <= 65535, A > 0, 0 <= G <= %d", kMaxG);
    FRCNN_REQUIRE(anchors && reg && label, "frcnn_anchor_target_finish: null pointer");
    const int Gp = G > 0 ? G : 1;
    AtWs w = carve_at(workspace, N, A, Gp);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_anchor_target_finish: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(samp_emit_kernel<0>, dim3(2 * N), dim3(kSampThreads), 0, st, w.calls, w.jrec, w.pos_list,
                       w.neg_list, A, w.keep, nullptr, 0);
    FRCNN_LAUNCH_CHECK("samp_emit_kernel");
    const int nblk = (A + 255) / 256;
    hipLaunchKernelGGL(at_finish_kernel, dim3(nblk, N), dim3(256), 0, st, anchors, A, w.gt, w.gcount,
                       Gp, w.row_arg, w.label0, w.keep, w.sampled, label, reg);
    FRCNN_LAUNCH_CHECK("at_finish_kernel");
    if (argmax && hipMemcpyAsync(argmax, w.row_arg, sizeof(int32_t) * N * A,
                                 hipMemcpyDeviceToDevice, st) != hipSuccess)
        return check_launch("frcnn_anchor_target_finish copy");
    if (max_iou && hipMemcpyAsync(max_iou, w.row_max, sizeof(double) * N * A,
                                  hipMemcpyDeviceToDevice, st) != hipSuccess)
        return check_launch("frcnn_anchor_target_finish copy");
    return FRCNN_OK;
}

extern "C" int frcnn_anchor_target_sample(int N, int A, int G, const float* anchors, int n_sample,
                                          double pos_ratio, uint32_t* rng_state, double* reg,
                                          int32_t* label, int32_t* argmax, double* max_iou,
                                          void* workspace, size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(anchors && reg && label, "frcnn_anchor_target_sample: null pointer");
    const int rc = frcnn_anchor_target_draw(N, A, G, n_sample, pos_ratio, rng_state, workspace, ws_bytes, stream);
    if (rc != FRCNN_OK) return rc;
    return frcnn_anchor_target_finish(N, A, G, anchors, reg, label, argmax, max_iou, workspace, ws_bytes, stream);
}

extern "C" int frcnn_anchor_target(int N, int A, int G, const float* anchors, const double* boxes,
                                   const double* labels, int n_sample, double pos_iou_thresh,
                                   double neg_iou_thresh, double pos_ratio, uint32_t* rng_state,
                                   double* reg, int32_t* label, int32_t* argmax, double* max_iou,
                                   void* workspace, size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(anchors && reg && label, "frcnn_anchor_target: null pointer");
    const int n_pos_max = static_cast<int>(pos_ratio * n_sample);
    FRCNN_REQUIRE(n_sample - (n_pos_max < 0 ? 0 : n_pos_max) <= kMaxKeep && n_pos_max <= kMaxKeep,
                  "frcnn_anchor_target: n_sample too large");
    int rc = frcnn_anchor_target_prepare(N, A, G, anchors, boxes, labels, pos_iou_thresh, neg_iou_thresh,
                                         workspace, ws_bytes, stream);
    if (rc != FRCNN_OK) return rc;
    return frcnn_anchor_target_sample(N, A, G, anchors, n_sample, pos_ratio, rng_state, reg, label, argmax,
                                      max_iou, workspace, ws_bytes, stream);
}

namespace {
struct PtWs {
    double* gt;
    double* gl;
    int* gcount;
    double* roi_all;
    int32_t* assign;
    int* pos_list;
    int* neg_list;
    int* npos;
    int* nneg;
    int* sample;
    int* spos;
    int4* calls;
    int* jrec;
    DrawCap cap;
    DrawBufs draw;
    size_t bytes;
};
PtWs carve_pt(void* ws, int N, int Rp, int Gp, int n_sample) {
    Carver c(ws);
    PtWs w{};
    const size_t stride = static_cast<size_t>(Rp) + Gp;
    w.gt = c.take<double>(static_cast<size_t>(N) * Gp * 4);
    w.gl = c.take<double>(static_cast<size_t>(N) * Gp);
    w.gcount = c.take<int>(N);
    w.roi_all = c.take<double>(N * stride * 4);
    w.assign = c.take<int32_t>(N * stride);
    w.pos_list = c.take<int>(N * stride);
    w.neg_list = c.take<int>(N * stride);
    w.npos = c.take<int>(N);
    w.nneg = c.take<int>(N);
    w.sample = c.take<int>(static_cast<size_t>(N) * n_sample);
    w.spos = c.take<int>(N);
    w.calls = c.take<int4>(2 * N);
    w.jrec = c.take<int>(static_cast<size_t>(2 * N) * kMaxKeep);
    w.cap = draw_cap(N, static_cast<int64_t>(N) * static_cast<int64_t>(stride));
    w.draw = carve_draw(c, w.cap);
    w.bytes = c.used();
    return w;
}

void pt_ops(const PtWs& w, int N, int stride, int n_sample, int pos_per_image, int32_t* sample_count, DrawOps& ops,
            SerialPt& pt) {
    ops.n_pt = N;
    ops.pt_n_sample = n_sample;
    ops.pt_pos_per_image = pos_per_image;
    ops.pt_npos = w.npos;
    ops.pt_nneg = w.nneg;
    ops.pt_calls = w.calls;
    ops.pt_scount = sample_count;
    ops.pt_spos = w.spos;
    ops.pt_jrec = w.jrec;
    pt = SerialPt{N, stride, n_sample, pos_per_image, w.pos_list, w.neg_list, w.npos, w.nneg, sample_count, w.spos,
                  w.calls, w.jrec};
}
}  // namespace

extern "C" size_t frcnn_proposal_target_workspace_size(int N, int Rp, int G, int n_sample) {
    if (N <= 0 || Rp < 0 || G < 0 || n_sample <= 0) return 0;
    return carve_pt(nullptr, N, Rp, G > 0 ? G : 1, n_sample).bytes;
}

extern "C" int frcnn_proposal_target_prepare(int N, int Rp, const float* rois, const int32_t* rcount, int G,
                                             const double* boxes, const double* labels, int n_sample,
                                             double pos_iou_thresh, double neg_iou_thresh_high,
                                             double neg_iou_thresh_low, void* workspace, size_t ws_bytes,
                                             void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && Rp >= 0 && G >= 0 && G <= kMaxG && n_sample > 0,
                  "frcnn_proposal_target_prepare: bad shape");
    FRCNN_REQUIRE(Rp + G <= kMaxKeep, "frcnn_proposal_target_prepare: rois + gt must be <= %d", kMaxKeep);
    FRCNN_REQUIRE(rcount, "frcnn_proposal_target_prepare: null pointer");
    FRCNN_REQUIRE(Rp == 0 || rois, "frcnn_proposal_target_prepare: null rois");
    FRCNN_REQUIRE(G == 0 || (boxes && labels), "frcnn_proposal_target_prepare: null boxes");
    const int Gp = G > 0 ? G : 1;
    PtWs w = carve_pt(workspace, N, Rp, Gp, n_sample);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_proposal_target_prepare: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    hipStream_t st = as_stream(stream);
    if (G > 0) {
        hipLaunchKernelGGL(gt_compact_kernel, dim3(N), dim3(64), 0, st, boxes, labels, G, w.gt, w.gl,
                           w.gcount);
        FRCNN_LAUNCH_CHECK("gt_compact_kernel");
    } else if (hipMemsetAsync(w.gcount, 0, sizeof(int) * N, st) != hipSuccess) {
        return check_launch("frcnn_proposal_target memset");
    }
    hipLaunchKernelGGL(pt_iou_kernel, dim3(N), dim3(1024), 0, st, rois, rcount, Rp, w.gt, w.gl,
                       w.gcount, Gp, pos_iou_thresh, neg_iou_thresh_high, neg_iou_thresh_low,
                       w.roi_all, w.assign, w.pos_list, w.neg_list, w.npos, w.nneg);
    FRCNN_LAUNCH_CHECK("pt_iou_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_proposal_target_draw(int N, int Rp, int G, int n_sample, double pos_ratio, uint32_t* rng_state,
                                          int32_t* sample_count, void* workspace, size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && Rp >= 0 && G >= 0 && G <= kMaxG && n_sample > 0,
                  "frcnn_proposal_target_draw: bad shape");
    // the recorded swaps of one choice() call fill one [kMaxKeep] row of jrec
    FRCNN_REQUIRE(Rp + G <= kMaxKeep, "frcnn_proposal_target_draw: rois + gt must be <= %d", kMaxKeep);
    FRCNN_REQUIRE(rng_state && sample_count, "frcnn_proposal_target_draw: null pointer");
    const int Gp = G > 0 ? G : 1;
    PtWs w = carve_pt(workspace, N, Rp, Gp, n_sample);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_proposal_target_draw: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    hipStream_t st = as_stream(stream);
    const int stride = Rp + Gp;
    const int pos_per_image = static_cast<int>(std::nearbyint(n_sample * pos_ratio));  // np.round
    DrawOps ops{};
    SerialPt pt{};
    pt_ops(w, N, stride, n_sample, pos_per_image, sample_count, ops, pt);
    return launch_draws(ops, nullptr, &pt, rng_state, w.cap, w.draw, st);
}

extern "C" int frcnn_target_draws(int N, int A, int G_at, int n_sample_at, double pos_ratio_at, void* at_workspace,
                                  size_t at_bytes, int Rp, int G_pt, int n_sample_pt, double pos_ratio_pt,
                                  void* pt_workspace, size_t pt_bytes, int32_t* sample_count, uint32_t* rng_state,
                                  void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && A > 0 && G_at >= 0 && G_at <= kMaxG && Rp >= 0 && G_pt >= 0 &&
                      G_pt <= kMaxG && n_sample_pt > 0 && n_sample_at > 0,
                  "frcnn_target_draws: bad shape");
    const int n_pos_max = static_cast<int>(pos_ratio_at * n_sample_at);
    FRCNN_REQUIRE(n_sample_at - (n_pos_max < 0 ? 0 : n_pos_max) <= kMaxKeep && n_pos_max <= kMaxKeep,
                  "frcnn_target_draws: n_sample_at must be in 1..%d per choice() call", kMaxKeep);
    FRCNN_REQUIRE(Rp + G_pt <= kMaxKeep, "frcnn_target_draws: rois + gt must be <= %d", kMaxKeep);
    FRCNN_REQUIRE(rng_state && sample_count, "frcnn_target_draws: null pointer");
    AtWs aw = carve_at(at_workspace, N, A, G_at > 0 ? G_at : 1);
    FRCNN_REQUIRE(at_workspace && at_bytes >= aw.bytes, "frcnn_target_draws: anchor workspace %zu < %zu", at_bytes,
                  aw.bytes);
    const int Gp = G_pt > 0 ? G_pt : 1;
    PtWs pw = carve_pt(pt_workspace, N, Rp, Gp, n_sample_pt);
    FRCNN_REQUIRE(pt_workspace && pt_bytes >= pw.bytes, "frcnn_target_draws: proposal workspace %zu < %zu", pt_bytes,
                  pw.bytes);
    const int pos_per_image = static_cast<int>(std::nearbyint(n_sample_pt * pos_ratio_pt));  // np.round
    DrawOps ops{};
    SerialAt at{};
    SerialPt pt{};
    at_ops(aw, N, A, n_sample_at, n_pos_max, ops, at);
    pt_ops(pw, N, Rp + Gp, n_sample_pt, pos_per_image, sample_count, ops, pt);
    return launch_draws(ops, &at, &pt, rng_state, aw.cap, aw.draw, as_stream(stream));
}

extern "C" int frcnn_proposal_target_draw_status(int N, int Rp, int G, int n_sample, const void* workspace,
                                                 size_t ws_bytes, int* out) {
    FRCNN_REQUIRE(N > 0 && Rp >= 0 && G >= 0 && n_sample > 0 && out, "frcnn_proposal_target_draw_status: bad argument");
    PtWs w = carve_pt(const_cast<void*>(workspace), N, Rp, G > 0 ? G : 1, n_sample);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_proposal_target_draw_status: workspace too small");
    return draw_status(w.draw, w.cap, out);
}

extern "C" int frcnn_proposal_target_finish(int N, int Rp, int G, int n_sample, const double* reg_mean,
                                            const double* reg_std, const int32_t* sample_count,
                                            double* sample_roi, double* gt_roi_reg, double* gt_roi_label,
                                            void* workspace, size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(N > 0 && N <= 65535 && Rp >= 0 && G >= 0 && G <= kMaxG && n_sample > 0,
                  "frcnn_proposal_target_finish: bad shape");
    FRCNN_REQUIRE(Rp + G <= kMaxKeep, "frcnn_proposal_target_finish: rois + gt must be <= %d", kMaxKeep);
    FRCNN_REQUIRE(sample_roi && gt_roi_reg && gt_roi_label && sample_count && reg_mean && reg_std,
                  "frcnn_proposal_target_finish: null pointer");
    const int Gp = G > 0 ? G : 1;
    PtWs w = carve_pt(workspace, N, Rp, Gp, n_sample);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_proposal_target_finish: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    hipStream_t st = as_stream(stream);
    const int stride = Rp + Gp;
    hipLaunchKernelGGL(samp_emit_kernel<1>, dim3(2 * N), dim3(kSampThreads), 0, st, w.calls, w.jrec, w.pos_list,
                       w.neg_list, stride, nullptr, w.sample, n_sample);
    FRCNN_LAUNCH_CHECK("samp_emit_kernel");
    RegNorm nrm;
    for (int c = 0; c < 4; ++c) {
        nrm.mean[c] = reg_mean[c];
        nrm.stdv[c] = reg_std[c];
    }
    hipLaunchKernelGGL(pt_finish_kernel, dim3(N, (n_sample + 127) / 128), dim3(128), 0, st, stride,
                       n_sample, w.roi_all, w.assign, w.gt, w.gl, w.gcount, Gp, w.sample, sample_count,
                       w.spos, nrm, sample_roi, gt_roi_reg, gt_roi_label);
    FRCNN_LAUNCH_CHECK("pt_finish_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_proposal_target_sample(int N, int Rp, int G, int n_sample, double pos_ratio,
                                            const double* reg_mean, const double* reg_std,
                                            uint32_t* rng_state, double* sample_roi, double* gt_roi_reg,
                                            double* gt_roi_label, int32_t* sample_count, void* workspace,
                                            size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(sample_roi && gt_roi_reg && gt_roi_label && reg_mean && reg_std,
                  "frcnn_proposal_target_sample: null pointer");
    const int rc = frcnn_proposal_target_draw(N, Rp, G, n_sample, pos_ratio, rng_state, sample_count, workspace,
                                              ws_bytes, stream);
    if (rc != FRCNN_OK) return rc;
    return frcnn_proposal_target_finish(N, Rp, G, n_sample, reg_mean, reg_std, sample_count, sample_roi,
                                        gt_roi_reg, gt_roi_label, workspace, ws_bytes, stream);
}

extern "C" int frcnn_proposal_target(int N, int Rp, const float* rois, const int32_t* rcount, int G,
                                     const double* boxes, const double* labels, int n_sample,
                                     double pos_ratio, double pos_iou_thresh,
                                     double neg_iou_thresh_high, double neg_iou_thresh_low,
                                     const double* reg_mean, const double* reg_std,
                                     uint32_t* rng_state, double* sample_roi, double* gt_roi_reg,
                                     double* gt_roi_label, int32_t* sample_count, void* workspace,
                                     size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(rng_state && sample_roi && gt_roi_reg && gt_roi_label && sample_count && reg_mean && reg_std,
                  "frcnn_proposal_target: null pointer");
    const int rc = frcnn_proposal_target_prepare(N, Rp, rois, rcount, G, boxes, labels, n_sample, pos_iou_thresh,
                                                 neg_iou_thresh_high, neg_iou_thresh_low, workspace, ws_bytes,
                                                 stream);
    if (rc != FRCNN_OK) return rc;
    return frcnn_proposal_target_sample(N, Rp, G, n_sample, pos_ratio, reg_mean, reg_std, rng_state, sample_roi,
                                        gt_roi_reg, gt_roi_label, sample_count, workspace, ws_bytes, stream);
}

extern "C" int frcnn_bbox_iou(const void* a, int a_is_f64, int64_t na, const void* b, int b_is_f64,
                              int64_t nb, void* out, void* stream) {
    FRCNN_REQUIRE(na >= 0 && nb >= 0, "frcnn_bbox_iou: bad shape");
    if (na == 0 || nb == 0) return FRCNN_OK;
    FRCNN_REQUIRE(a && b && out, "frcnn_bbox_iou: null pointer");
    const int64_t tot = na * nb;
    dim3 grid(static_cast<unsigned>((tot + 255) / 256));
    hipStream_t st = as_stream(stream);
    if (!a_is_f64 && !b_is_f64)
        hipLaunchKernelGGL((bbox_iou_kernel<float, float, float>), grid, dim3(256), 0, st,
                           static_cast<const float*>(a), na, static_cast<const float*>(b), nb,
                           static_cast<float*>(out));
    else if (!a_is_f64)
        hipLaunchKernelGGL((bbox_iou_kernel<float, double, double>), grid, dim3(256), 0, st,
                           static_cast<const float*>(a), na, static_cast<const double*>(b), nb,
                           static_cast<double*>(out));
    else if (!b_is_f64)
        hipLaunchKernelGGL((bbox_iou_kernel<double, float, double>), grid, dim3(256), 0, st,
                           static_cast<const double*>(a), na, static_cast<const float*>(b), nb,
                           static_cast<double*>(out));
    else
        hipLaunchKernelGGL((bbox_iou_kernel<double, double, double>), grid, dim3(256), 0, st,
                           static_cast<const double*>(a), na, static_cast<const double*>(b), nb,
                           static_cast<double*>(out));
    FRCNN_LAUNCH_CHECK("bbox_iou_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_bbox2reg(const void* anchors, int a_is_f64, const void* bbox, int b_is_f64,
                              int64_t n, double* out, void* stream) {
    FRCNN_REQUIRE(n >= 0, "frcnn_bbox2reg: n < 0");
    if (n == 0) return FRCNN_OK;
    FRCNN_REQUIRE(anchors && bbox && out, "frcnn_bbox2reg: null pointer");
    dim3 grid(static_cast<unsigned>((n + 255) / 256));
    hipStream_t st = as_stream(stream);
    if (!a_is_f64 && !b_is_f64)
        hipLaunchKernelGGL((bbox2reg_kernel<float, float>), grid, dim3(256), 0, st,
                           static_cast<const float*>(anchors), static_cast<const float*>(bbox), n, out);
    else if (!a_is_f64)
        hipLaunchKernelGGL((bbox2reg_kernel<float, double>), grid, dim3(256), 0, st,
                           static_cast<const float*>(anchors), static_cast<const double*>(bbox), n, out);
    else if (!b_is_f64)
        hipLaunchKernelGGL((bbox2reg_kernel<double, float>), grid, dim3(256), 0, st,
                           static_cast<const double*>(anchors), static_cast<const float*>(bbox), n, out);
    else
        hipLaunchKernelGGL((bbox2reg_kernel<double, double>), grid, dim3(256), 0, st,
                           static_cast<const double*>(anchors), static_cast<const double*>(bbox), n, out);
    FRCNN_LAUNCH_CHECK("bbox2reg_kernel");
    return FRCNN_OK;
}



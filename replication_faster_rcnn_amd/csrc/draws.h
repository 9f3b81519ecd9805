// Chip-wide draws: the choice() calls of a target creator as chunk functions
// (round 4).  Included by targets.hip inside namespace frcnn (uses mt_temper,
// mask_for, mt_mix, kMtN, kMtM, kMaxKeep).
//
// The calls of one op (AnchorTarget: per image the positive then the negative
// choice(); ProposalTarget likewise, utils/utils.py:190-202, 248-258) consume
// numpy's MT19937 stream back to back.  Their Fisher-Yates steps form one
// sequence of states (call k, step i), i = i_hi(k) .. 1; a word w met in state
// (k, i) is accepted iff (w & mask(i)) <= i, which moves to (k, i - 1) (to the
// next call's first step after i = 1).  Instead of walking that sequence word
// by word on one CU:
//  * draw_twist_kernel twists every state block the op can need (its expected
//    length + 12 sigma) into a flat word buffer (one workgroup, one barrier per
//    624-word block);
//  * draw_chunk_kernel (one wave per 64-word chunk of the stream, chip-wide)
//    builds, for every mask region the chunk's entering state can plausibly be
//    in (the expected step count at the chunk's offset +- 3 sqrt(words) + 96),
//    the chunk's exact function of the entering step:
//      - region steps [lo, hi] (mask hi = 2^b - 1, lo >= 64): word t is
//        accepted iff the entering step i_in >= tau_t (acceptance only grows
//        with i_in inside a region), tau_t = v_t + #{s < t : u_s <= v_t} with
//        u_s = tau_s - rank(tau_s), every u_s > v_t dropping by one when v_t is
//        inserted (tools/proto_thresholds.py checks this against the serial
//        walk for every i_in); a path that leaves the region continues from
//        the exact step lo - 1 at the word after its (i_in - lo + 1)-th
//        acceptance, so a 64-entry crossing table (lane t: the exit state of
//        the suffix that starts at word t + 1 in state (k, lo - 1), walked
//        serially across any further regions and call ends) completes it;
//      - steps 1..63: a candidate table (lane j: the exit state of the whole
//        chunk entered in step lo + j, walked serially);
//  * draw_chain_kernel carries the exact state through the chunks in order:
//    per chunk one compare + ballot + popcount against the matching entry
//    (prefetched by three helper waves into an LDS ring), a serial walk of the
//    chunk only when no entry matches;
//  * draw_replay_kernel (one lane per chunk, chip-wide) re-walks the chunks
//    whose steps are recorded from the chain's exact entering states and
//    writes the swaps J into jrec exactly like the one-workgroup sampler, and
//    the chain writes numpy's final state (the block of the last consumed word
//    + pos), so samp_emit_kernel and the callers see the same outputs.
// A state is packed as k << 22 | i; k == nc (all calls done) carries the
// chunk-relative index just past the last consumed word in the low bits.

constexpr int kDrawChunk = 64;
constexpr int kDrawEnt = 12;          // directory entries (and pool slots) per chunk
constexpr int kIBits = 22;
constexpr uint32_t kIMask = (1u << kIBits) - 1u;
constexpr uint32_t kDrawNone = 0xffffffffu;
enum : uint32_t { kEntThr = 1u, kEntCand = 2u, kEntCross = 4u };

__device__ __forceinline__ uint32_t dstate(uint32_t k, uint32_t i) { return (k << kIBits) | i; }

struct DrawSeg {      // a mask region of one call, in stream order
    double w0;        // expected words consumed before it
    int k, ia, ib;    // call, first (highest) and last step
    int mask;         // 2^b - 1
};

struct DrawHdr {      // device-side plan and results of one op
    int nc;           // calls that consume words
    int nseg;
    int nchunks;      // chunks with directories
    int nblocks;      // blocks in the word buffer (block 0 = the incoming state)
    int p0;           // numpy's pos at entry
    int used_chunks;  // chunks the chain walked (for the replay)
    int consumed;     // words consumed by the op
    int status;       // 0 ok; 1 the word buffer ran out; 2 a directory pool overflow (slow path taken)
    int fallbacks;    // chunks walked serially by the chain
    int pool_next;    // entry data slots handed out
    int total_steps;
    int pad;
    unsigned long long prof[8];  // -DFRCNN_DRAW_PROF: chain cycles (total, waiting, hit path, slow walks)
};
#ifdef FRCNN_DRAW_PROF
#define DPROF_T() __builtin_amdgcn_s_memtime()
#else
#define DPROF_T() 0ull
#endif

struct DrawWs {       // carved from the target creator's workspace
    DrawHdr* hdr;
    int* c_ihi;       // [2N] first step of each word-consuming call
    int* c_rlo;       // [2N] lowest recorded step (J[i - rlo] for i >= rlo)
    int* c_slot;      // [2N] jrec row
    int* c_u0;        // [2N + 1] steps before the call
    DrawSeg* seg;     // [2N * 24]
    uint32_t* words;  // [nblk_max * 624] untempered state blocks, flat (absolute word index)
    uint4* dir;       // [chunks_max * kDrawEnt] (s_lo, s_hi, kind, data slot)
    uint32_t* pool;   // [chunks_max * kDrawEnt][128]
    uint32_t* sin;    // [chunks_max] entering state of every walked chunk
    int nblk_max, chunks_max;
};

// harmonic number H(n) (n >= 0), for the expected words of a region (a guess:
// single precision)
__device__ __forceinline__ float harm(float n) {
    if (n < 1.0f) return 0.0f;
    if (n < 8.0f) {
        float s = 0.0f;
        for (int j = 1; j <= static_cast<int>(n); ++j) s += 1.0f / j;
        return s;
    }
    return __logf(n) + 0.5772157f + 0.5f / n - 1.0f / (12.0f * n * n);
}

constexpr int kPlanThreads = 64;
constexpr int kPlanMaxCalls = 1 << (32 - kIBits);  // the state packs the call index in 10 bits

// After thread 0 wrote the call list (c_ihi / c_rlo / c_slot, hdr->nc): the
// steps before every call, the mask regions with their expected word counts
// (a thread per call, then a serial prefix), and how many words / blocks /
// chunks the op can need (expected + 12 sigma, sigma^2 <= 2 * steps since every
// step accepts with probability >= 1/2).  All kPlanThreads threads.
__device__ void draw_plan_tail(DrawWs w, int p0) {
    __shared__ int seg_off[kPlanMaxCalls + 1];
    __shared__ float call_w[kPlanMaxCalls];
    __shared__ double call_w0[kPlanMaxCalls + 1];
    DrawHdr* h = w.hdr;
    const int nc = h->nc;
    if (threadIdx.x == 0) {
        int u = 0, ns = 0;
        for (int k = 0; k < nc; ++k) {
            w.c_u0[k] = u;
            seg_off[k] = ns;
            const int ihi = w.c_ihi[k];
            u += ihi;
            ns += 32 - __builtin_clz(static_cast<uint32_t>(ihi));
        }
        w.c_u0[nc] = u;
        seg_off[nc] = ns;
        h->nseg = ns;
        h->total_steps = u;
    }
    __syncthreads();
    // expected words per call (a thread per call), a serial prefix in LDS, then
    // every region's start
    for (int k = threadIdx.x; k < nc; k += kPlanThreads) {
        const int ihi = w.c_ihi[k];
        float t = 0.0f;
        for (int b = 32 - __builtin_clz(static_cast<uint32_t>(ihi)); b >= 1; --b) {
            const int mask = static_cast<int>((1u << b) - 1u);
            const int ia = ihi < mask ? ihi : mask, ib = 1 << (b - 1);
            t += (mask + 1.0f) * (harm(ia + 1.0f) - harm(static_cast<float>(ib)));
        }
        call_w[k] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double acc = 0.0;
        for (int k = 0; k < nc; ++k) {
            call_w0[k] = acc;
            acc += call_w[k];
        }
        call_w0[nc] = acc;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nc; k += kPlanThreads) {
        const int ihi = w.c_ihi[k];
        int sidx = seg_off[k];
        double w0 = call_w0[k];
        for (int b = 32 - __builtin_clz(static_cast<uint32_t>(ihi)); b >= 1; --b, ++sidx) {
            const int mask = static_cast<int>((1u << b) - 1u);
            const int ia = ihi < mask ? ihi : mask, ib = 1 << (b - 1);
            DrawSeg sg;
            sg.w0 = w0;
            sg.k = k;
            sg.ia = ia;
            sg.ib = ib;
            sg.mask = mask;
            w.seg[sidx] = sg;
            w0 += (mask + 1.0f) * (harm(ia + 1.0f) - harm(static_cast<float>(ib)));
        }
    }
    if (threadIdx.x != 0) return;
    const int u = w.c_u0[nc];
    const double need = call_w0[nc] + 12.0 * sqrt(2.0 * u) + 256.0;
    int nch = static_cast<int>(need / kDrawChunk) + 1;
    if (u == 0) nch = 0;
    int nblk = (p0 + nch * kDrawChunk + kMtN - 1) / kMtN + 1;
    if (nblk > w.nblk_max) nblk = w.nblk_max;
    if ((nblk * kMtN - p0) / kDrawChunk < nch) nch = (nblk * kMtN - p0) / kDrawChunk;
    if (nch > w.chunks_max) nch = w.chunks_max;
    h->nchunks = nch;
    h->nblocks = nblk;
    h->p0 = p0;
    h->used_chunks = 0;
    h->consumed = 0;
    h->status = 0;
    h->fallbacks = 0;
    h->pool_next = 0;
}

// AnchorTarget's calls (at_sample_kernel's order and outputs)
__global__ __launch_bounds__(kPlanThreads) void draw_plan_at_kernel(int N, int n_sample, int n_pos_max,
                                                                   const int* __restrict__ npos,
                                                                   const int* __restrict__ nneg,
                                                                   const uint32_t* __restrict__ rng,
                                                                   int* __restrict__ sampled,
                                                                   int4* __restrict__ calls, DrawWs w) {
    __shared__ int2 pq[kPlanMaxCalls / 2];
    for (int n = threadIdx.x; n < N; n += kPlanThreads) pq[n] = make_int2(npos[n], nneg[n]);
    __syncthreads();
    if (threadIdx.x == 0) {
        int nc = 0;
        for (int n = 0; n < N; ++n) {
            const int P = pq[n].x, Q = pq[n].y;
            const int pos_after = P > n_pos_max ? n_pos_max : P;
            for (int call = 0; call < 2; ++call) {
                const int cnt = call == 0 ? P : Q;
                const int m = call == 0 ? n_pos_max : n_sample - pos_after;
                const bool do_call = cnt > m;
                const int k = cnt - m;
                sampled[2 * n + call] = do_call ? 1 : 0;
                calls[2 * n + call] = do_call ? make_int4(cnt, k, cnt, 0) : make_int4(0, 0, 0, 0);
                if (do_call && cnt >= 2) {
                    w.c_ihi[nc] = cnt - 1;
                    w.c_rlo[nc] = k;
                    w.c_slot[nc] = 2 * n + call;
                    ++nc;
                }
            }
        }
        w.hdr->nc = nc;
    }
    __syncthreads();
    draw_plan_tail(w, static_cast<int>(rng[kMtN]));
}

// ProposalTarget's calls (pt_sample_kernel's order and outputs)
__global__ __launch_bounds__(kPlanThreads) void draw_plan_pt_kernel(int N, int n_sample, int pos_per_image,
                                                                   const int* __restrict__ npos,
                                                                   const int* __restrict__ nneg,
                                                                   const uint32_t* __restrict__ rng,
                                                                   int* __restrict__ scount, int* __restrict__ spos,
                                                                   int4* __restrict__ calls, DrawWs w) {
    __shared__ int2 pq[kPlanMaxCalls / 2];
    for (int n = threadIdx.x; n < N; n += kPlanThreads) pq[n] = make_int2(npos[n], nneg[n]);
    __syncthreads();
    if (threadIdx.x == 0) {
        int nc = 0;
        for (int n = 0; n < N; ++n) {
            const int P = pq[n].x, Q = pq[n].y;
            const int kp = P < pos_per_image ? P : pos_per_image;
            int kn = n_sample - kp;
            kn = Q < kn ? Q : kn;
            for (int call = 0; call < 2; ++call) {
                const int cnt = call == 0 ? P : Q;
                const int k = call == 0 ? kp : kn;
                const int off = call == 0 ? 0 : kp;
                calls[2 * n + call] = cnt > 0 ? make_int4(cnt, 1, k, off) : make_int4(0, 0, 0, 0);
                if (cnt >= 2) {
                    w.c_ihi[nc] = cnt - 1;
                    w.c_rlo[nc] = 1;
                    w.c_slot[nc] = 2 * n + call;
                    ++nc;
                }
            }
            scount[n] = kp + kn;
            spos[n] = kp;
        }
        w.hdr->nc = nc;
    }
    __syncthreads();
    draw_plan_tail(w, static_cast<int>(rng[kMtN]));
}

// Block 0 = the incoming state; block b + 1 = the twist of block b (numpy's
// mt19937_gen), into the flat buffer.  One workgroup of 256 threads; the
// current block stays in LDS (two slots), one barrier per block.
__global__ __launch_bounds__(256) void draw_twist_kernel(const uint32_t* __restrict__ rng, DrawWs w) {
    __shared__ uint32_t blk[2][kMtN];
    const int nb = w.hdr->nblocks;
    for (int i = threadIdx.x; i < kMtN; i += 256) {
        const uint32_t v = rng[i];
        blk[0][i] = v;
        w.words[i] = v;
    }
    __syncthreads();
    for (int b = 1; b < nb; ++b) {
        const uint32_t* old = blk[(b - 1) & 1];
        uint32_t* nw = blk[b & 1];
        uint32_t* g = w.words + static_cast<size_t>(b) * kMtN;
        const int t = threadIdx.x;
        if (t < kMtN - kMtM) {
            const uint32_t a = old[t + kMtM] ^ mt_mix(old[t], old[t + 1]);
            const uint32_t c = a ^ mt_mix(old[t + 227], old[t + 228]);
            nw[t] = a;
            nw[t + 227] = c;
            g[t] = a;
            g[t + 227] = c;
            if (t + 454 < kMtN - 1) {
                const uint32_t d = c ^ mt_mix(old[t + 454], old[t + 455]);
                nw[t + 454] = d;
                g[t + 454] = d;
            } else if (t + 454 == kMtN - 1) {
                const uint32_t n0 = old[kMtM] ^ mt_mix(old[0], old[1]);
                const uint32_t d = c ^ mt_mix(old[kMtN - 1], n0);
                nw[kMtN - 1] = d;
                g[kMtN - 1] = d;
            }
        }
        __syncthreads();
    }
}

// One step of the serial automaton on lane state s with tempered word x; the
// call table in c_ihi.  t = the chunk-relative index of the word (for k == nc).
__device__ __forceinline__ uint32_t draw_step(uint32_t s, uint32_t x, int t, int nc, const int* c_ihi) {
    const uint32_t k = s >> kIBits;
    if (static_cast<int>(k) >= nc) return s;
    uint32_t i = s & kIMask;
    if ((x & mask_for(i)) <= i) {
        if (--i == 0) {
            const uint32_t k1 = k + 1;
            return static_cast<int>(k1) < nc ? dstate(k1, static_cast<uint32_t>(c_ihi[k1]))
                                             : dstate(k1, static_cast<uint32_t>(t + 1));
        }
        return dstate(k, i);
    }
    return s;
}

// Serial walk of the chunk's words t >= start(lane) from lane state s.
__device__ __forceinline__ uint32_t draw_walk(uint32_t s, int start, uint32_t x_lane, int nc, const int* c_ihi) {
    for (int t = 0; t < kDrawChunk; ++t) {
        const uint32_t x = __builtin_amdgcn_readlane(x_lane, t);
        if (t >= start) s = draw_step(s, x, t, nc, c_ihi);
    }
    return s;
}

// One wave per chunk: the directory of entries for the mask regions its
// entering state can plausibly be in (the kDrawEnt nearest the expected state,
// in stream order), entry e's data in pool slot c * kDrawEnt + e.
__global__ __launch_bounds__(256) void draw_chunk_kernel(DrawWs w) {
    const int lane = threadIdx.x & 63;
    const int c = static_cast<int>(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const DrawHdr* h = w.hdr;
    if (c >= h->nchunks) return;
    const int nc = h->nc, nseg = h->nseg, p0 = h->p0;
    uint4* dir = w.dir + static_cast<size_t>(c) * kDrawEnt;
    const uint32_t x = mt_temper(w.words[static_cast<size_t>(p0) + static_cast<size_t>(c) * kDrawChunk + lane]);
    // expected steps done after g words: invert the regions' expected word counts
    const float g = static_cast<float>(c) * kDrawChunk;
    int lo_s = 0, hi_s = nseg - 1;  // last segment with w0 <= g
    while (lo_s < hi_s) {
        const int mid = (lo_s + hi_s + 1) >> 1;
        if (w.seg[mid].w0 <= g) lo_s = mid; else hi_s = mid - 1;
    }
    const DrawSeg sg = w.seg[lo_s];
    float ig = (sg.ia + 1.5f) * __expf(-(g - static_cast<float>(sg.w0)) / (sg.mask + 1.0f)) - 0.5f;
    if (ig < sg.ib) ig = static_cast<float>(sg.ib);
    if (ig > sg.ia) ig = static_cast<float>(sg.ia);
    const int ihk = w.c_ihi[sg.k];
    const int ug = w.c_u0[sg.k] + (ihk - static_cast<int>(ig));
    const int R = static_cast<int>(3.0f * sqrtf(g)) + 96;
    const int total = h->total_steps;
    int ulo = ug - R, uhi = ug + R;
    if (ulo < 0) ulo = 0;
    if (uhi > total - 1) uhi = total - 1;
    // candidate entries in stream order (lane e: state range and kind), and the
    // one holding the guess
    uint32_t e_lo = kDrawNone, e_hi = 0, e_kind = 0;
    int ne = 0, eg = -1;
    if (ulo <= uhi) {
        int k0 = sg.k;
        while (k0 > 0 && w.c_u0[k0] > ulo) --k0;
        for (int k = k0; k < nc && ne < 64; ++k) {
            const int u0 = w.c_u0[k], ihi = w.c_ihi[k];
            if (u0 > uhi) break;
            if (u0 + ihi - 1 < ulo) continue;
            const int imax = ihi - ((ulo > u0 ? ulo : u0) - u0);
            const int imin = ihi - ((uhi < u0 + ihi - 1 ? uhi : u0 + ihi - 1) - u0);
            const int ig_k = (k == sg.k) ? static_cast<int>(ig) : -1;
            for (int b = 32 - __builtin_clz(static_cast<uint32_t>(imax)); b >= 7 && ne < 64; --b) {
                const int lo = 1 << (b - 1), hi = (1 << b) - 1;
                const int a = imin > lo ? imin : lo, z = imax < hi ? imax : hi;
                if (a > z) continue;
                const uint32_t kind = kEntThr | (a < lo + kDrawChunk ? kEntCross : 0u);
                if (lane == ne) {
                    e_lo = dstate(k, a);
                    e_hi = dstate(k, z);
                    e_kind = kind;
                }
                if (ig_k >= lo && ig_k <= hi) eg = ne;
                ++ne;
            }
            if (imin < 64 && ne < 64) {
                const int a = imin > 1 ? imin : 1, z = imax < 63 ? imax : 63;
                if (a <= z) {
                    if (lane == ne) {
                        e_lo = dstate(k, a);
                        e_hi = dstate(k, z);
                        e_kind = kEntCand;
                    }
                    if (ig_k >= 1 && ig_k < 64) eg = ne;
                    ++ne;
                }
            }
        }
    }
    // keep the kDrawEnt entries nearest the guess
    int first = 0;
    if (ne > kDrawEnt) {
        first = (eg < 0 ? ne / 2 : eg) - kDrawEnt / 2;
        if (first < 0) first = 0;
        if (first > ne - kDrawEnt) first = ne - kDrawEnt;
    }
    const int nkeep = ne - first < kDrawEnt ? ne - first : kDrawEnt;
    for (int j = 0; j < nkeep; ++j) {
        const uint32_t slo = __builtin_amdgcn_readlane(e_lo, first + j);
        const uint32_t shi = __builtin_amdgcn_readlane(e_hi, first + j);
        const uint32_t kind = __builtin_amdgcn_readlane(e_kind, first + j);
        const uint32_t k = slo >> kIBits, a = slo & kIMask, z = shi & kIMask;
        uint32_t* d = w.pool + (static_cast<size_t>(c) * kDrawEnt + j) * 128;
        if (kind & kEntThr) {
            const uint32_t hi = mask_for(a), lo = (hi >> 1) + 1u;
            // thresholds: insert v_t in stream order
            const uint32_t v = x & hi;
            uint32_t u = 0x7fffffffu, tau = 0;
            for (int t = 0; t < kDrawChunk; ++t) {
                const uint32_t vt = __builtin_amdgcn_readlane(v, t);
                const uint64_t le = __ballot(u <= vt);
                const uint32_t kk = static_cast<uint32_t>(__popcll(le));
                u -= (u > vt) ? 1u : 0u;
                if (lane == t) {
                    u = vt;
                    tau = vt + kk;
                }
            }
            d[lane] = tau;
            if (kind & kEntCross) d[64 + lane] = draw_walk(dstate(k, lo - 1), lane + 1, x, nc, w.c_ihi);
        } else {
            const uint32_t s0 = lane <= static_cast<int>(z - a) ? dstate(k, a + lane) : dstate(nc, 0);
            d[lane] = draw_walk(s0, 0, x, nc, w.c_ihi);
        }
        if (lane == 0) dir[j] = make_uint4(slo, shi, kind, 0u);
    }
    if (lane >= nkeep && lane < kDrawEnt) dir[lane] = make_uint4(kDrawNone, 0u, 0u, 0u);
}

// The exact state through the chunks.  Wave 0 carries it; waves 1..15 stage the
// chunks into an LDS ring, kGroup chunks per step: for each chunk only the (at
// most kSlotEnt) directory entries its entering state can fall in -- the ones
// nearest the state the chain last published, advanced by the expected steps
// to the chunk (+- 4 sigma) -- with their data laid out [lane][entry], so the
// chain reads a chunk with three LDS reads issued two chunks ahead.  A state
// outside them reads the chunk's whole directory from global memory; a chunk
// without a matching entry is walked serially.
constexpr int kChainRing = 32;  // (a power of two: slot = c & 31)
constexpr int kChainWaves = 16;
constexpr int kStagers = 12;  // waves off SIMD 0 (wave w runs on SIMD w % 4)
constexpr int kSlotEnt = 4;
constexpr int kGroup = 4;
struct ChainSlot {
    uint4 dir[kSlotEnt];
    uint4 tau[64];  // [lane]: entries 0..3
    uint4 crs[64];
};
struct ChainLds {
    ChainSlot slot[kChainRing];
    int seq[kChainRing];  // chunk index + 1 held by the slot
    int pos;              // chunks the chain has finished
    int stop;
    uint32_t s_pub;       // the state entering chunk pos (a prediction input)
    int ihi[kPlanMaxCalls];
    int u0[kPlanMaxCalls + 1];
};

__device__ __forceinline__ int lds_acq(const int* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ int lds_rlx(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_rel(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_put(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// resolve chunk c from its entering state s with entry e's data (tau, cross)
__device__ __forceinline__ uint32_t chain_apply(uint32_t s, uint32_t kind, uint32_t elo, uint32_t tv, uint32_t xv,
                                                int lane) {
    const uint32_t k = s >> kIBits, i = s & kIMask;
    if (kind & kEntCand) return __builtin_amdgcn_readlane(tv, static_cast<int>(i - (elo & kIMask)));
    const uint32_t lo = (mask_for(i) >> 1) + 1u;
    const uint64_t acc = __ballot(tv <= i);
    const uint32_t nb = static_cast<uint32_t>(__popcll(acc & 0x7fffffffffffffffull));
    if (nb <= i - lo) return dstate(k, i - static_cast<uint32_t>(__popcll(acc)));
    // the (i - lo + 1)-th acceptance leaves the region; the rest from (k, lo - 1)
    const uint32_t before = static_cast<uint32_t>(__builtin_amdgcn_mbcnt_hi(
        static_cast<uint32_t>(acc >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(acc), 0u)));
    const uint64_t at = __ballot(((acc >> lane) & 1ull) && before == i - lo);
    const int t = __ffsll(static_cast<unsigned long long>(at)) - 1;
    return __builtin_amdgcn_readlane(xv, t);
}

// expected step index after `words` more words from state sp: within a mask
// region (steps lo..hi, mask M) j words take step i to (i + 1) exp(-j / (M + 1)) - 1
__device__ float predict_u(uint32_t sp, float words, int nc, const int* ihi, const int* u0) {
    int k = static_cast<int>(sp >> kIBits);
    float i = static_cast<float>(sp & kIMask);
    for (int it = 0; it < 48 && k < nc; ++it) {
        const uint32_t ii = static_cast<uint32_t>(i);
        const float M1 = static_cast<float>(mask_for(ii)) + 1.0f, lo = M1 * 0.5f;
        // words to leave the region: (M + 1) ln((i + 1) / lo)
        const float wl = M1 * __logf((i + 1.0f) / lo);
        if (words < wl) {
            i = (i + 1.0f) * __expf(-words / M1) - 1.0f;
            break;
        }
        words -= wl;
        i = lo - 1.0f;
        if (i < 1.0f) {
            if (++k >= nc) break;
            i = static_cast<float>(ihi[k]);
        }
    }
    if (k >= nc) return static_cast<float>(u0[nc]);
    return static_cast<float>(u0[k] + ihi[k]) - i;
}

__device__ __forceinline__ uint32_t pick4(uint4 v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

// the chunk's whole directory and data from global memory (the slow path)
__device__ uint32_t chain_global(const DrawWs& w, int c, uint32_t s, int lane, int nc, bool& walked) {
    const uint4 d = lane < kDrawEnt ? w.dir[static_cast<size_t>(c) * kDrawEnt + lane]
                                    : make_uint4(kDrawNone, 0u, 0u, 0u);
    const uint64_t hit = __ballot(lane < kDrawEnt && d.x != kDrawNone && d.x <= s && s <= d.y);
    walked = !hit;
    if (hit) {
        const int e = __ffsll(static_cast<unsigned long long>(hit)) - 1;
        const uint32_t* src = w.pool + (static_cast<size_t>(c) * kDrawEnt + e) * 128;
        return chain_apply(s, __builtin_amdgcn_readlane(d.z, e), __builtin_amdgcn_readlane(d.x, e), src[lane],
                           src[64 + lane], lane);
    }
    const uint32_t x = mt_temper(w.words[static_cast<size_t>(w.hdr->p0) + static_cast<size_t>(c) * kDrawChunk + lane]);
    return draw_walk(s, 0, x, nc, w.c_ihi);
}

__global__ __launch_bounds__(kChainWaves * 64) void draw_chain_kernel(uint32_t* __restrict__ rng, DrawWs w) {
    __shared__ ChainLds L;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    DrawHdr* h = w.hdr;
    const int nch = h->nchunks, nc = h->nc, p0 = h->p0;
    for (int t = threadIdx.x; t < kChainRing; t += kChainWaves * 64) L.seq[t] = 0;
    for (int k = threadIdx.x; k <= nc; k += kChainWaves * 64) {
        L.u0[k] = w.c_u0[k];
        if (k < nc) L.ihi[k] = w.c_ihi[k];
    }
    const uint32_t s_init = nc > 0 ? dstate(0, static_cast<uint32_t>(w.c_ihi[0])) : dstate(0, 0);
    if (threadIdx.x == 0) {
        L.pos = 0;
        L.stop = 0;
        L.s_pub = s_init;
    }
    __syncthreads();
    if (wid > 0) {
        // stagers: the waves off the chain's SIMD (waves 4, 8, 12 share SIMD 0
        // with wave 0 and retire), chunk group g = chunks kGroup g .. + kGroup - 1
        if ((wid & 3) == 0) return;
        const int sid = wid - 1 - (wid >> 2);  // 0 .. kStagers - 1
        const int seg = lane / kDrawEnt, ent = lane % kDrawEnt;  // lanes 0..47: (chunk of the group, entry)
        for (int g = sid; g * kGroup < nch; g += kStagers) {
            const int c0 = g * kGroup;
            const int cc = c0 + seg;
            const bool lv = seg < kGroup && cc < nch;
            const uint4 d = lv ? w.dir[static_cast<size_t>(cc) * kDrawEnt + ent] : make_uint4(kDrawNone, 0u, 0u, 0u);
            for (int spin = 0;; ++spin) {  // ring space (bounded: a lost chain stops the op, not the GPU)
                if (lds_rlx(&L.stop) || spin > (1 << 22)) break;
                if (lds_rlx(&L.pos) > c0 + kGroup - 1 - kChainRing) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (lds_rlx(&L.stop)) break;
            // predicted step index of each lane's chunk, and each entry's distance to it
            const int pc = lds_rlx(&L.pos);
            const uint32_t sp = static_cast<uint32_t>(lds_rlx(reinterpret_cast<const int*>(&L.s_pub)));
            const float dist = static_cast<float>(cc - pc > 0 ? cc - pc : 0);
            const float upred = predict_u(sp, dist * kDrawChunk, nc, L.ihi, L.u0);
            uint32_t key = 0xffffffffu;
            if (lv && d.x != kDrawNone) {
                const uint32_t k = d.x >> kIBits;
                const float ub = static_cast<float>(L.u0[k] + L.ihi[k]);
                const float ulo = ub - static_cast<float>(d.y & kIMask), uhi = ub - static_cast<float>(d.x & kIMask);
                const float gap = upred < ulo ? ulo - upred : upred > uhi ? upred - uhi : 0.0f;
                const float W = 4.0f * sqrtf(dist * 16.0f) + 24.0f;
                if (gap <= W) key = (static_cast<uint32_t>(gap) << 8) | static_cast<uint32_t>(lane);
            }
            // per chunk of the group: the kSlotEnt nearest entries
            uint32_t tv[kGroup][kSlotEnt], xv[kGroup][kSlotEnt];
            uint4 dv[kGroup];  // lane q: entry q of chunk j
#pragma unroll
            for (int j = 0; j < kGroup; ++j) {
                uint32_t kk = seg == j ? key : 0xffffffffu;
                dv[j] = make_uint4(kDrawNone, 0u, 0u, 0u);
#pragma unroll
                for (int q = 0; q < kSlotEnt; ++q) {
                    const uint32_t m = __ockl_wfred_min_u32(kk);
                    tv[j][q] = 0u;
                    xv[j][q] = 0u;
                    if (m != 0xffffffffu) {
                        const int l = static_cast<int>(m & 0xffu);
                        if (lane == l) kk = 0xffffffffu;
                        const uint32_t kind = __builtin_amdgcn_readlane(d.z, l);
                        if (lane == q)
                            dv[j] = make_uint4(__builtin_amdgcn_readlane(d.x, l), __builtin_amdgcn_readlane(d.y, l), kind, 0u);
                        const uint32_t* src = w.pool + (static_cast<size_t>(c0 + j) * kDrawEnt + (l - j * kDrawEnt)) * 128;
                        tv[j][q] = src[lane];
                        if (kind & kEntCross) xv[j][q] = src[64 + lane];
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kGroup; ++j) {
                const int c = c0 + j;
                if (c >= nch) break;
                ChainSlot& S = L.slot[c % kChainRing];
                if (lane < kSlotEnt) S.dir[lane] = dv[j];
                S.tau[lane] = make_uint4(tv[j][0], tv[j][1], tv[j][2], tv[j][3]);
                S.crs[lane] = make_uint4(xv[j][0], xv[j][1], xv[j][2], xv[j][3]);
                if (lane == 0) lds_rel(&L.seq[c % kChainRing], c + 1);
            }
        }
        return;
    }
    // wave 0: the chain
    bool ok = nc == 0, lost = false;
    uint32_t s = s_init;
    int c = 0, consumed = 0, fb = 0, slow = 0;
    unsigned long long nspin = 0, nstall = 0;
    auto wait_seq = [&](int cc) {
        int spin = 0;
        while (lds_acq(&L.seq[cc & (kChainRing - 1)]) != cc + 1 && ++spin < (1 << 22)) __builtin_amdgcn_s_sleep(0);
        if (spin >= (1 << 22)) lost = true;
        nspin += spin;
        nstall += spin ? 1 : 0;
    };
    uint4 dA = make_uint4(kDrawNone, 0u, 0u, 0u), tA = make_uint4(0u, 0u, 0u, 0u), xA = tA;
    uint4 dB = dA, tB = tA, xB = tA;
    if (!ok && nch > 0) {
        wait_seq(0);
        const ChainSlot& S = L.slot[0];
        dA = S.dir[lane & (kSlotEnt - 1)];
        tA = S.tau[lane];
        xA = S.crs[lane];
    }
    if (!ok && nch > 1) {
        wait_seq(1);
        const ChainSlot& S = L.slot[1];
        dB = S.dir[lane & (kSlotEnt - 1)];
        tB = S.tau[lane];
        xB = S.crs[lane];
    }
    __builtin_amdgcn_s_setprio(3);
    int sq = nch > 2 ? lds_rlx(&L.seq[2]) : 0;  // chunk c + 2's slot, read one chunk early
    // One step: chunk c + 2's slot into set Z, chunk c resolved from set X
    // (set Y holds chunk c + 1).  The loop is unrolled three times with the sets
    // rotating X -> Y -> Z, so no registers move between steps.
    auto step = [&](uint4& dX, uint4& tX, uint4& xX, uint4& dZ, uint4& tZ, uint4& xZ) {
        if (c + 2 < nch) {
            if (sq != c + 3) wait_seq(c + 2);
            const ChainSlot& S = L.slot[(c + 2) & (kChainRing - 1)];
            dZ = S.dir[lane & (kSlotEnt - 1)];
            tZ = S.tau[lane];
            xZ = S.crs[lane];
            if (c + 3 < nch) sq = lds_rlx(&L.seq[(c + 3) & (kChainRing - 1)]);
        }
#ifndef FRCNN_DRAW_DBG
        if (lane == 0) w.sin[c] = s;
#endif
        // the entry holding s (lanes >= kSlotEnt mirror 0..3; an empty entry's
        // s_lo = kDrawNone exceeds every state), then its function of s
        const uint64_t hit = __builtin_amdgcn_ballot_w64(dX.x <= s && s <= dX.y);
        uint32_t ns;
        if (hit) {
            const int e = static_cast<int>(__builtin_amdgcn_readfirstlane(__ffsll(static_cast<unsigned long long>(hit)) - 1));
            const uint32_t kind = __builtin_amdgcn_readlane(dX.z, e);
            const uint32_t tv = pick4(tX, e), i = s & kIMask;
            if (kind & kEntCand) {
                ns = __builtin_amdgcn_readlane(tv, static_cast<int>(i - (__builtin_amdgcn_readlane(dX.x, e) & kIMask)));
            } else {
                const uint32_t lo = (mask_for(i) >> 1) + 1u;
                const uint64_t acc = __builtin_amdgcn_ballot_w64(tv <= i);
                const uint32_t n = static_cast<uint32_t>(__popcll(acc));
                if (n - static_cast<uint32_t>(acc >> 63) <= i - lo) {
                    ns = s - n;  // (k, i - n): i - n >= lo - 1 >= 63
                } else {  // the (i - lo + 1)-th acceptance leaves the region; the rest from (k, lo - 1)
                    const uint32_t before = __builtin_amdgcn_mbcnt_hi(
                        static_cast<uint32_t>(acc >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(acc), 0u));
                    const uint64_t at = __builtin_amdgcn_ballot_w64(((acc >> lane) & 1ull) && before == i - lo);
                    ns = __builtin_amdgcn_readlane(pick4(xX, e), __ffsll(static_cast<unsigned long long>(at)) - 1);
                }
            }
        } else {
            bool walked = false;
            ns = chain_global(w, c, s, lane, nc, walked);
            ++slow;
            fb += walked ? 1 : 0;
        }
        s = __builtin_amdgcn_readfirstlane(ns);
#ifdef FRCNN_DRAW_DBG
        if ((c & 3) == 3) {
#else
        {
#endif
            lds_put(reinterpret_cast<int*>(&L.s_pub), static_cast<int>(s));
            lds_put(&L.pos, c + 1);
        }
        if (static_cast<int>(s >> kIBits) >= nc) {
            consumed = c * kDrawChunk + static_cast<int>(s & kIMask);
            ok = true;
        }
        ++c;
        return ok || lost || c >= nch;
    };
    uint4 dC = dA, tC = tA, xC = xA;
    if (!ok && nch > 0) {
        for (;;) {
            if (step(dA, tA, xA, dC, tC, xC)) break;
            if (step(dB, tB, xB, dA, tA, xA)) break;
            if (step(dC, tC, xC, dB, tB, xB)) break;
        }
    }
    lds_rel(&L.stop, 1);
    if (lane == 0) {
        h->used_chunks = c;
        h->consumed = consumed;
        h->fallbacks = fb;
        h->pool_next = slow;
        if (!ok) atomicMax(&h->status, lost ? 3 : 1);
        h->prof[4] = nspin;
        h->prof[5] = nstall;
    }
    // numpy's state after the op: the block of the last consumed word, pos past it
    if (ok && consumed > 0) {
        const int a = p0 + consumed - 1;
        const int b = a / kMtN;
        for (int j = lane; j < kMtN; j += 64) rng[j] = w.words[static_cast<size_t>(b) * kMtN + j];
        if (lane == 0) rng[kMtN] = static_cast<uint32_t>(a - b * kMtN + 1);
    }
}

// One lane per walked chunk: the recorded swaps of the steps it holds.
__global__ __launch_bounds__(256) void draw_replay_kernel(int* __restrict__ jrec, DrawWs w) {
    const DrawHdr* h = w.hdr;
    const int c = static_cast<int>(blockIdx.x * 256 + threadIdx.x);
    if (c >= h->used_chunks) return;
    const int nc = h->nc;
    uint32_t s = w.sin[c];
    uint32_t k = s >> kIBits, i = s & kIMask;
    if (static_cast<int>(k) >= nc) return;
    if (static_cast<int>(i) < w.c_rlo[k] && i > kDrawChunk) return;  // nothing recorded within reach
    const uint32_t* wp = w.words + static_cast<size_t>(h->p0) + static_cast<size_t>(c) * kDrawChunk;
    int rlo = w.c_rlo[k];
    int* jr = jrec + static_cast<size_t>(w.c_slot[k]) * kMaxKeep;
    for (int t = 0; t < kDrawChunk; ++t) {
        const uint32_t v = mt_temper(wp[t]) & mask_for(i);
        if (v <= i) {
            if (static_cast<int>(i) >= rlo) jr[i - rlo] = static_cast<int>(v);
            if (--i == 0) {
                if (static_cast<int>(++k) >= nc) return;
                i = static_cast<uint32_t>(w.c_ihi[k]);
                rlo = w.c_rlo[k];
                jr = jrec + static_cast<size_t>(w.c_slot[k]) * kMaxKeep;
            }
        }
    }
}

// ROUND-2 EXPERIMENT (not built): block-sorted RoIPool forward.  Measured on
// MI355X (tools/ab_roi_pool.py, profiles/r2_roi_pool_experiments.md): cfg2 145 us
// vs 81 us for the dense kernel and 68.5 us for the wave-per-RoI kernel -- the
// (image, window width) units fragment each block (~35 units per 27 RoIs), the
// per-unit overhead keeps VALU at 34 M instructions, and the block barriers
// expose the unit / record load latency (SQ_WAIT_ANY 2.9x).  Kept as a record;
// the host side lived in roi_pool.hip (sb_plan / sb_launch) at commit time.
// --------------------------------------------------- block-sorted forward
// The default forward, for RoIs grouped by image.  RoIs are cut into blocks
// of RB consecutive RoIs.
//   roi_block_sort_kernel (one 256-thread workgroup per block, once per call):
//     every bin's window [hs, hs+dh) x [ws, ws+dw) (nets/heads.py:48,
//     torchvision's bin arithmetic); bins counting-sorted by (image, dw
//     descending, dh ascending) and cut into units of <= 64 bins of ONE image
//     and ONE window width (dh may differ by the odd row: a unit walks its
//     largest dh, shorter windows repeat their last row, which can never pass
//     the strict '>' again); with the head transform (nets/heads.py:42-47),
//     the [idx, box] rows are written here.
//   roi_pool_fwd_blk_kernel (workgroup = CG channel planes of one image,
//     staged once into LDS, NaN -> -inf, and a share of the image's blocks):
//     waves pull the block's units -- the window width is wave-uniform, so
//     the walk is scalar-controlled and unrolled for dw <= 4 with the pixel
//     offsets as LDS immediates, and no lane walks a wider window than its
//     own (a RoI-per-wave mapping walks every lane through the RoI's largest
//     window, 1.5x the pixels on VOC-shaped RoIs, and idles 15 of 64 lanes);
//     the (max, argmax) pairs go to an LDS staging image of the block; the
//     block then leaves as contiguous 16-B stores (RoI r's channels
//     [c0, c0+CG) x PH*PW are one run of out / argmax).
// Windows wider than 14 or taller than 15 columns / rows take per-lane
// walks; RoIs with an out-of-range batch index are written by grid row N.
constexpr int kSbMaxRB = 64;
constexpr int kSbNormal = 0, kSbEmpty = 1, kSbLarge = 2;

struct SbWs {
    int2* recs;    // [nblk][RB*PHW]: { RoI, k | hs << 6 | ws << 16 | dh << 26 }
    int4* units;   // [nblk][ucap]:  { first record, image, count | dw << 8 | maxdh << 12 | kind << 16, - }
    int* nunits;   // [nblk]
};
__host__ __device__ constexpr int sb_ucap(int rb, int phw) { return (rb * phw + 63) / 64 + 16 * rb; }

template <int NT, bool HEAD>
__global__ __launch_bounds__(NT) void roi_block_sort_kernel(const float* __restrict__ rois, int R, int N, int H,
                                                            int W, int PH, int PW, float ss, int RB, SbWs ws,
                                                            HeadArgs hd) {
    extern __shared__ __attribute__((aligned(16))) int s_hist[];  // [nimg * 256] (keys), then scan
    __shared__ int4 s_geo[kSbMaxRB];
    __shared__ int s_img[kSbMaxRB];   // image slot of each RoI (-1: out-of-range batch index)
    __shared__ int s_bidx[kSbMaxRB];  // batch index of each image slot
    __shared__ int s_nimg, s_nu;
    __shared__ int s_red[NT / 64];
    const int j = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int PHW = PH * PW;
    const int r0 = j * RB;
    const int nb = min(RB, R - r0);
    // ---- RoIs: geometry, batch index, image slots (RoIs are grouped by image)
    if (tid < 64) {
        int bi = -1;
        if (tid < nb) {
            const int r = r0 + tid;
            float bx[5];
            if (HEAD) {
                head_box(rois, hd, r, bx);
                if (hd.boxes) {
#pragma unroll
                    for (int q = 0; q < 5; ++q) hd.boxes[static_cast<size_t>(r) * 5 + q] = bx[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 5; ++q) bx[q] = rois[static_cast<size_t>(r) * 5 + q];
            }
            const RoiGeom gm = roi_geom(bx, ss, PH, PW);
            s_geo[tid] = make_int4(gm.sh, gm.sw, __float_as_int(gm.bh), __float_as_int(gm.bw));
            bi = static_cast<int>(bx[0]);
        }
        const int prev = __shfl_up(bi, 1, 64);
        const bool start = tid < nb && (tid == 0 || prev != bi);
        const uint64_t st = __ballot(start);
        const int slot = static_cast<int>(__popcll(st & ((2ull << tid) - 1))) - 1;  // starts at or before tid
        if (tid < nb) s_img[tid] = (bi >= 0 && bi < N) ? slot : -1;
        if (start) s_bidx[slot] = bi;
        if (tid == 0) s_nimg = static_cast<int>(__popcll(st));
    }
    __syncthreads();
    const int nimg = s_nimg;
    const int nkeys = nimg * 256;
    for (int i = tid; i < nkeys; i += NT) s_hist[i] = 0;
    __syncthreads();
    // ---- bins: key = slot*256 + (15 - dwk)*16 + dhk; dwk 1..14 normal, 0 empty, 15 large
    auto bin_key = [&](int t, uint32_t& rec) {
        const int i = t / PHW, k = t - (t / PHW) * PHW;
        const int sl = s_img[i];
        if (sl < 0) return -1;
        const int4 gq = s_geo[i];
        RoiGeom gm;
        gm.sh = gq.x;
        gm.sw = gq.y;
        gm.bh = __int_as_float(gq.z);
        gm.bw = __int_as_float(gq.w);
        const int ph = k / PW;
        const int4 g = geom_bin(gm, H, W, ph, k - ph * PW);
        const int dh = g.y - g.x, dw = g.w - g.z;
        int dwk, dhk;
        if (dh <= 0 || dw <= 0) {
            dwk = 0;
            dhk = 0;
        } else if (dh > 15 || dw > 14) {
            dwk = 15;
            dhk = 0;
        } else {
            dwk = dw;
            dhk = dh;
        }
        rec = static_cast<uint32_t>(k) | (static_cast<uint32_t>(g.x) << 6) | (static_cast<uint32_t>(g.z) << 16) |
              (static_cast<uint32_t>(dhk) << 26);
        return sl * 256 + (15 - dwk) * 16 + dhk;
    };
    const int nbin = nb * PHW;
    for (int t0 = 0; t0 < nbin; t0 += NT) {  // histogram: one LDS atomic per (wave, key)
        const int t = t0 + tid;
        uint32_t rec;
        const int key = t < nbin ? bin_key(t, rec) : -1;
        uint64_t todo = __ballot(key >= 0);
        while (todo) {
            const int l = __ffsll(static_cast<unsigned long long>(todo)) - 1;
            const int lk = __builtin_amdgcn_readlane(key, l);
            const uint64_t m = __ballot(key == lk);
            if (lane == l) atomicAdd(&s_hist[lk], static_cast<int>(__popcll(m)));
            todo &= ~m;
        }
    }
    __syncthreads();
    // ---- exclusive scan of the histogram (per thread a contiguous run of keys)
    const int per = (nkeys + NT - 1) / NT;
    const int k0 = tid * per, k1 = min(k0 + per, nkeys);
    int loc = 0;
    for (int q = k0; q < k1; ++q) loc += s_hist[q];
    int inc = loc;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) s_red[wid] = inc;
    __syncthreads();
    int run = inc - loc;
    for (int w = 0; w < wid; ++w) run += s_red[w];
    for (int q = k0; q < k1; ++q) {
        const int c = s_hist[q];
        s_hist[q] = run;  // becomes the key's record cursor
        run += c;
    }
    if (tid == 0) s_nu = 0;
    __syncthreads();
    // ---- scatter the records (same key order as the histogram pass)
    int2* recs = ws.recs + static_cast<size_t>(j) * RB * PHW;
    for (int t0 = 0; t0 < nbin; t0 += NT) {
        const int t = t0 + tid;
        uint32_t rec = 0;
        const int key = t < nbin ? bin_key(t, rec) : -1;
        uint64_t todo = __ballot(key >= 0);
        int pos = 0;
        while (todo) {
            const int l = __ffsll(static_cast<unsigned long long>(todo)) - 1;
            const int lk = __builtin_amdgcn_readlane(key, l);
            const uint64_t m = __ballot(key == lk);
            int base = 0;
            if (lane == l) base = atomicAdd(&s_hist[lk], static_cast<int>(__popcll(m)));
            base = __builtin_amdgcn_readlane(base, l);
            if (key == lk) pos = base + static_cast<int>(__popcll(m & lanemask_lt()));
            todo &= ~m;
        }
        if (key >= 0) recs[pos] = make_int2(r0 + t / PHW, static_cast<int>(rec));
    }
    __syncthreads();
    // ---- units: per (image slot, dwk) group, in key order; s_hist[key] now = end of the key
    int4* units = ws.units + static_cast<size_t>(j) * sb_ucap(RB, PHW);
    const int ngroups = nimg * 16;
    for (int g = tid; g < ngroups; g += NT) {
        const int gb = g * 16;
        const int start = gb == 0 ? 0 : s_hist[gb - 1];
        const int endg = s_hist[gb + 15];
        const int cnt = endg - start;
        if (cnt <= 0) continue;
        const int dwk = 15 - (g & 15);
        const int kind = dwk == 0 ? kSbEmpty : dwk == 15 ? kSbLarge : kSbNormal;
        const int nu = (cnt + 63) >> 6;
        const int u0 = atomicAdd(&s_nu, nu);  // unit order inside a block does not matter for the outputs
        for (int q = 0; q < nu; ++q) {
            const int cu = min(64, cnt - 64 * q);
            const int last = start + 64 * q + cu - 1;
            const int maxdh = (static_cast<uint32_t>(recs[last].y) >> 26) & 15;
            units[u0 + q] = make_int4(static_cast<int>(j * RB * PHW + start + 64 * q), s_bidx[g >> 4],
                                      cu | (dwk << 8) | (maxdh << 12) | (kind << 16), 0);
        }
    }
    __syncthreads();
    if (tid == 0) ws.nunits[j] = s_nu;
}

// Strict-'>' first-max update of CG running (max, index) pairs with the pixel
// pair (a, b) (b after a in row-major order, or a repeat): m' = max3(m, a, b);
// the index moves iff m' > m, to a if a == m'.
template <int CG>
__device__ __forceinline__ void bs_pair(const float4* __restrict__ q4, int HWs, int a, int b, float (&mv)[CG],
                                        int (&mi)[CG]) {
    constexpr int NP = CG / 4;
    float4 va[NP], vb[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        va[q] = q4[q * HWs + a];
        vb[q] = q4[q * HWs + b];
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const float a4[4] = {va[q].x, va[q].y, va[q].z, va[q].w};
        const float b4[4] = {vb[q].x, vb[q].y, vb[q].z, vb[q].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 4 * q + j;
            const float m = max3_raw(mv[c], a4[j], b4[j]);
            const int ip = a4[j] == m ? a : b;
            mi[c] = m > mv[c] ? ip : mi[c];
            mv[c] = m;
        }
    }
}

// Walk of a unit of window width DW (compile time): rows 0 .. maxdh-1
// (uniform); a lane's rows past its own dh repeat its last row.  Odd DW pairs
// pixels across two rows.
template <int CG, int DW>
__device__ __forceinline__ void blk_scan_dw(const float4* __restrict__ q4, int HWs, int W, int pix0, int dh,
                                            int maxdh, float (&mv)[CG], int (&mi)[CG]) {
    if (DW % 2 == 0) {
        for (int i = 0; i < maxdh; ++i) {
            const int p = pix0 + min(i, dh - 1) * W;
#pragma unroll
            for (int c = 0; c < DW; c += 2) bs_pair<CG>(q4, HWs, p + c, p + c + 1, mv, mi);
        }
    } else {
        for (int i = 0; i < maxdh; i += 2) {
            const int p0 = pix0 + min(i, dh - 1) * W, p1 = pix0 + min(i + 1, dh - 1) * W;
#pragma unroll
            for (int t = 0; t < 2 * DW; t += 2) {
                const int a = t < DW ? p0 + t : p1 + (t - DW);
                const int b = t + 1 < DW ? p0 + t + 1 : p1 + (t + 1 - DW);
                bs_pair<CG>(q4, HWs, a, b, mv, mi);
            }
        }
    }
}

template <int NT, int CG, bool HEAD>
__global__ __launch_bounds__(NT) void roi_pool_fwd_blk_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const float* __restrict__ boxes5, int R,
    int C, int H, int W, int PH, int PW, float ss, int RB, SbWs ws, float* __restrict__ out,
    int32_t* __restrict__ argmax, HeadArgs hd) {
    constexpr int NP = CG / 4;
    extern __shared__ __attribute__((aligned(16))) float4 q4[];
    __shared__ int s_red[2 * (NT / 64)];
    __shared__ int s_ua, s_ub, s_next;
    const int PHW = PH * PW;
    const int N = gridDim.y - 1;
    const int b = blockIdx.y, z = blockIdx.z, split = gridDim.z;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int HW = H * W;
    const int HWs = (HW + 15) & ~15;
    if (b == N) {  // out-of-range batch indices: [0, count(<0)) and [count(<N), R)
        const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, 0, N, s_red, 1)
                             : roi_range_sorted<NT>(rois, R, 0, N, s_red);
        const int n_lo = rg.x, tot = n_lo + (R - rg.y);
        const int lo = static_cast<int>(static_cast<int64_t>(tot) * z / split);
        const int hi = static_cast<int>(static_cast<int64_t>(tot) * (z + 1) / split);
        for (int e = lo * CG * PHW + tid; e < hi * CG * PHW; e += NT) {
            const int t = e / (CG * PHW);
            const int rem = e - t * (CG * PHW);
            const int r = t < n_lo ? t : rg.y + (t - n_lo);
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + rem;
            out[o] = 0.0f;
            argmax[o] = -1;
        }
        return;
    }
    const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, b, b + 1, s_red, 1)
                         : roi_range_sorted<NT>(rois, R, b, b + 1, s_red);
    if (rg.y <= rg.x) return;  // uniform
    const int jb0 = rg.x / RB, nblk = (rg.y - 1) / RB - jb0 + 1;
    const int ja = jb0 + static_cast<int>(static_cast<int64_t>(nblk) * z / split);
    const int jz = jb0 + static_cast<int>(static_cast<int64_t>(nblk) * (z + 1) / split);
    if (ja >= jz) return;  // uniform
    float* st_out = reinterpret_cast<float*>(q4 + NP * HWs);
    int32_t* st_am = reinterpret_cast<int32_t*>(st_out + static_cast<size_t>(RB) * CG * PHW);

    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    for (int p = tid; p < HW; p += NT) {
        float v[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            const float e = src[static_cast<size_t>(q) * HW + p];
            v[q] = e != e ? -INFINITY : e;
        }
#pragma unroll
        for (int k = 0; k < NP; ++k)
            q4[k * HWs + p] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    const int ucap = sb_ucap(RB, PHW);
    const int per4 = CG * PHW / 4;
    for (int j = ja; j < jz; ++j) {
        // ---- this image's units of block j (units of one image are not interleaved
        // with another's only by count: find them by image)
        if (tid == 0) {
            s_ua = 0x7fffffff;
            s_ub = 0;
            s_next = 0;
        }
        __syncthreads();  // tile staged / previous block flushed
        const int4* units = ws.units + static_cast<size_t>(j) * ucap;
        const int nu = ws.nunits[j];
        for (int u = tid; u < nu; u += NT)
            if (units[u].y == b) {
                atomicMin(&s_ua, u);
                atomicMax(&s_ub, u + 1);
            }
        __syncthreads();
        const int ua = s_ua, ub = s_ub;
        int ui = 0;
        if (lane == 0) ui = atomicAdd(&s_next, 1);
        ui = ua + __builtin_amdgcn_readfirstlane(ui);
        while (ui < ub) {
            int un = 0;
            if (lane == 0) un = atomicAdd(&s_next, 1);  // prefetch the next unit
            const int4 unit = units[ui];
            if (unit.y == b) {  // (uniform) units of other images inside [ua, ub) are skipped
                const int info = __builtin_amdgcn_readfirstlane(unit.z);
                const int cu = info & 255, dwk = (info >> 8) & 15, maxdh = (info >> 12) & 15, kind = info >> 16;
                const int2 rec = lane < cu ? ws.recs[unit.x + lane] : make_int2(-1, 0);
                const int r = rec.x;
                const uint32_t ry = static_cast<uint32_t>(rec.y);
                const int k = ry & 63;
                const int hs = (ry >> 6) & 1023, wsx = (ry >> 16) & 1023;
                const int dh = max(static_cast<int>((ry >> 26) & 15), 1);
                float mv[CG];
                int mi[CG];
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    mv[c] = kind == kSbEmpty ? 0.0f : -FLT_MAX;
                    mi[c] = -1;
                }
                if (kind == kSbLarge) {
                    if (r >= 0) {
                        const RoiGeom gm = roi_geom(boxes5 + static_cast<size_t>(r) * 5, ss, PH, PW);
                        const int ph = k / PW;
                        const int4 g = geom_bin(gm, H, W, ph, k - ph * PW);
                        for (int h = g.x; h < g.y; ++h)
                            for (int w = g.z; w < g.w; w += 2) {
                                const int a = h * W + w;
                                bs_pair<CG>(q4, HWs, a, h * W + min(w + 1, g.w - 1), mv, mi);
                            }
                    }
                } else if (kind == kSbNormal) {
                    const int pix0 = hs * W + wsx;
                    switch (dwk) {
                        case 1: blk_scan_dw<CG, 1>(q4, HWs, W, pix0, dh, maxdh, mv, mi); break;
                        case 2: blk_scan_dw<CG, 2>(q4, HWs, W, pix0, dh, maxdh, mv, mi); break;
                        case 3: blk_scan_dw<CG, 3>(q4, HWs, W, pix0, dh, maxdh, mv, mi); break;
                        case 4: blk_scan_dw<CG, 4>(q4, HWs, W, pix0, dh, maxdh, mv, mi); break;
                        default:
                            for (int i = 0; i < maxdh; ++i) {
                                const int p = pix0 + min(i, dh - 1) * W;
                                for (int c = 0; c < dwk; c += 2) bs_pair<CG>(q4, HWs, p + c, p + min(c + 1, dwk - 1), mv, mi);
                            }
                    }
                }
                // a zero maximum keeps the sign of the first max pixel (max3 may return +0)
                bool zero = false;
#pragma unroll
                for (int c = 0; c < CG; ++c) zero |= mv[c] == 0.0f && mi[c] >= 0;
                if (__ballot(zero)) {
#pragma unroll
                    for (int c = 0; c < CG; ++c)
                        if (mv[c] == 0.0f && mi[c] >= 0)
                            mv[c] = reinterpret_cast<const float*>(q4 + (c >> 2) * HWs + mi[c])[c & 3];
                }
                if (lane < cu) {
                    const int so = (r - j * RB) * CG * PHW + k;
#pragma unroll
                    for (int c = 0; c < CG; ++c) {
                        st_out[so + c * PHW] = mv[c];
                        st_am[so + c * PHW] = mi[c];
                    }
                }
            }
            ui = ua + __builtin_amdgcn_readfirstlane(un);
        }
        __syncthreads();
        // ---- the block's RoIs of this image: one contiguous run each (16-B stores)
        const int ra = max(rg.x, j * RB), rz = min(rg.y, (j + 1) * RB);
        const float4* so4 = reinterpret_cast<const float4*>(st_out);
        const int4* sa4 = reinterpret_cast<const int4*>(st_am);
        for (int e = tid; e < (rz - ra) * per4; e += NT) {
            const int i = e / per4, q = e - (e / per4) * per4;
            const int sl = ra - j * RB + i;
            const size_t g4 = ((static_cast<size_t>(ra + i) * C + c0) * PHW) / 4 + q;
            reinterpret_cast<float4*>(out)[g4] = so4[sl * per4 + q];
            reinterpret_cast<int4*>(argmax)[g4] = sa4[sl * per4 + q];
        }
    }
}


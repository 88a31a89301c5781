// Ray-tile engine (gfx950): per-ray compositing over the batched spherical geometry.
//
// It serves the two path C semantics the pair-major kernels of nlosgr_volume.hip cannot express,
// because both make a sample's value depend on the other Gaussians of the same ray:
//   * NLOSGR_MODE_OCCL — shared transmittance (volume_renderer.cu:80-137): per ray,
//       D_k = sum_g sigma_g pdf_g(x_k),  W_k = sum_g rho_g (1 - exp(-sigma_g pdf_g(x_k) c dT)),
//       T_k = exp(-c dT sum_{k'<k} D_k'),  out_k = T_k W_k, and 0 from the first T_k < 1e-4 on;
//   * NLOSGR_SELECT_AABB — path C's filter (ray_aabb.cu:10-61 + volume_renderer.cu:220-245): a ray
//       sums only the first 256 Gaussians, by index, whose 3-sigma box (bbox_compute.cuh) it hits,
//       each over the whole ray (cutoff <= 0: bins with m^2 <= kFullM2; beyond, pdf < 1e-39 underflows
//       anyway) or over its bins within the Mahalanobis cutoff (5.7: terms < 9e-8 of its peak dropped).
// With NLOSGR_SELECT_SUPPORT a ray sums every Gaussian over the bins within the Mahalanobis cutoff
// (dense when cutoff <= 0), as the pair-major kernels do.
//
// Work item = (wall point p, ray tile t): a TI x TJ block of the (theta, phi) ray grid, sized so
// the tile's [ray][bin] float2 rows fill 128 KB of LDS.  Persistent grid, one workgroup per CU
// (forward 16 waves, backward 8); slot s takes items s, s + nslot, ... (a static schedule, so every
// sum has a fixed order).
//   cull  : the waves test one Gaussian per lane per round against the tile's cone with
//           the bounding sphere of the support (or of the box); passing indices queue in LDS in
//           index order.
//   stage : 128 queued Gaussians at a time become pair records in LDS (A, u0 = A(p - mu), quadric
//           or box, sigma, rho = SH albedo of the view direction mu - p).
//   rays  : wave = ray.  Lane = staged Gaussian runs the ray test (quadric / slab + the 256 cap in
//           index order) and forms its 1-D Gaussian along the ray; then lane = bin: each 64-bin chunk
//           takes the entries overlapping it (ballot, in index order) and adds D and W into the
//           tile's rows (every lane owns its bin: no conflicts, no atomics).
//   scan  : wave = ray, lane = bin: exclusive wave scan of c dT D -> T, liveness, out = T W.
//           forward : sin(theta) out rows summed over the tile in row order -> partial histogram
//                     [p][t][nr]; tiles_reduce_kernel sums the tiles in order (x att x hscale).
//           backward: rows become (a, b) = (dL/dW, dL/dD), b from a suffix scan.
//   pairs : (backward) lane = (staged Gaussian, ray group) walks the in-support bins of its rays
//           reading (a, b) and accumulates the moments of dL/dpdf pdf; the four ray groups combine
//           in LDS in a fixed order; one 32-float record per (item, Gaussian) is added into the
//           slot's private accumulator row (plain read-modify-write).
//   finish: sums each Gaussian's slot rows in slot order and chains to the raw parameters.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nlosgr_common.hpp"

using namespace nlosgr;
using namespace nlosgr::detail;

namespace {

// threads per workgroup: forward 16 waves (one ray of a 16-ray tile each), backward 8 waves
// (its pair pass keeps more state per lane)
template <bool BWD>
constexpr int tile_threads() { return BWD ? 512 : 1024; }
constexpr int kWin = 128;              // staged Gaussians per window
#ifndef NLOSGR_TILES_DIAG_BUILD
#define NLOSGR_TILES_DIAG_BUILD 0          // per-phase cycle counters (a diagnostic build, NLOSGR_TILES_DIAG=1)
#endif
constexpr bool kDiag = NLOSGR_TILES_DIAG_BUILD;
constexpr int kStage = 20;             // floats per staged pair: A[9] u0[3] sel[6] sigma rho
constexpr int kRec = 32;               // floats per accumulator row: dA[9] dmu[3] dsigma pad[3] dF[16]
constexpr int kCap = NLOSGR_MAX_PER_RAY;
constexpr float kFullM2 = 180.0f;      // AABB selection: whole-ray support, pdf >= exp(-90)
constexpr float kLog2e = 1.44269504088896341f;
constexpr int kRowFloats = 32768;      // [ray][bin] float2 rows: 128 KB
constexpr int kList = 20;              // live entries per wave list pass (8 floats each)
#ifndef NLOSGR_CULL_U_BWD
#define NLOSGR_CULL_U_BWD 4
#endif
// cull: Gaussians per thread per round (one barrier pair per kCullU x threads); the forward's LDS holds 2
// (rows + stage + queue + lists: 157.5 of 160 KB), the backward's 8 waves leave room for 4
template <bool BWD>
constexpr int cull_u() { return BWD ? NLOSGR_CULL_U_BWD : 2; }
constexpr int kSlot = 6;               // backward pair slot: m0 m1 m2 dsigma drho | key
// support selection, backward: a block's live (entry, ray) pairs are walked in passes of 64 sorted by
// walk-length class (longest first) when there is more than one pass, so a pass's lanes walk similar
// lengths (a pass lasts as long as its longest walk).  C3 full-support occlusion backward 12.1 -> 10.8 s;
// not under AABB selection (3 % slower there, and the kernel is register-bound: it keeps the plain order)
constexpr int kWalkC0 = 96, kWalkC1 = 56, kWalkC2 = 28;   // walk-length class bounds (bins)
// backward pair walks (round 5; C3 occl AABB backward, one process per build on one box): sigma folded out of
// the loop with 1 - exp(-x) as a quartic in pdf 2532 -> 2291 ms (a diagnostic build with the polynomial cut
// to one multiply: -9 %, without the row reads: -2.6 %: the walks are VALU-bound), unrolled x4 (the row reads
// run ahead without register moves; x1 / 2 / 4 / 8: 2289 / 2229 / 2155 / 2146 ms, x8 spills) -> 2155, cubic
// instead of quartic -> 2123.  Measured and dropped: the exp2 recurrence re-seeded every 32 steps (a scalar
// branch per step: 2621 ms), or in 4-bin blocks (2131 ms), and forward rows without the per-bin support
// mask at cutoffs >= 5 (fwd 1283 vs 1260 ms masked), and two entries per forward loop iteration with both records
// read first (fwd 1335 vs 1260 ms; full support 6974 vs 6217), and a cubic 1 - exp(-x) in the forward rows
// (1268 vs 1265 ms: no gain)
#ifndef NLOSGR_TILE_OM3
#define NLOSGR_TILE_OM3 1
#endif
#ifndef NLOSGR_WALK_UNROLL
#define NLOSGR_WALK_UNROLL 4
#endif
#ifndef NLOSGR_WALK_RESEED
#define NLOSGR_WALK_RESEED 16   // backward pair walks: exp2 recurrence re-seeded every this many bins (0: exp2 per bin)
#endif
constexpr int kWalkReseed = NLOSGR_WALK_RESEED;
static_assert((kWalkReseed & (kWalkReseed - 1)) == 0, "the re-seed period is a power of two");
#ifndef NLOSGR_WALK_REC
#define NLOSGR_WALK_REC 1
#endif

struct TArgs {
    nlosgr_gaussians g;
    nlosgr_geometry geo;
    nlosgr_options opt;
    const GaussRec* recs;
    const float4* cull;      // [ng] (mu, bounding-sphere radius of the support / box)
    const float* bbox;       // [ng][6] (AABB selection)
    float* acc;              // [nslot][ng][kRec] (backward)
    float* hpart;            // [P][ntiles][nr] (forward)
    float* hist_out;
    float* ray_out;
    const float* grad_hist;
    const float* grad_ray;
    int ti, tj, rt;          // tile shape and rays per tile
    int ntile_i, ntile_j, ntiles;
    long long nitems;
    int nslot;
    unsigned long long* diag;   // NLOSGR_TILES_DIAG: per-phase cycles of thread 0, summed over workgroups
    int pbase;               // global index of wall point 0 of this launch (forward wall-point batches)
    unsigned long long* next;   // forward: dynamic item counter (items are independent; the backward keeps the
                                // static schedule, whose slot-private accumulator rows need a fixed order)
    float2* rcache;          // OCCL row cache [nitems][rt][nr] (D, W) (opt.ray_cache): the forward's rows,
                             // reloaded by the backward instead of re-running its first sweep
    const float* cones;      // [P][ntiles][8] tile cones of this launch's wall points (tile_cone_kernel)
    const unsigned long long* masks;   // tile bins [P][ntiles][nwords] (tile_bin_kernel), or null: cull in-kernel
    int nwords;              // 64-Gaussian words per tile bin row
};

__host__ __device__ inline int tile_rays(int nr) {
    int rt = 64;
    while (rt > 4 && 2 * rt * nr > kRowFloats) rt >>= 1;
    return rt;
}

struct TLayout {   // offsets in floats
    int rows, stage, queue, comb, misc, total;
    __host__ __device__ TLayout(int rt, int nr, int tb, bool bwd) {
        rows = 0;
        stage = rows + 2 * rt * nr;
        queue = stage + kWin * kStage;
        misc = queue + (bwd ? cull_u<true>() : cull_u<false>()) * tb + kWin;   // queue: one cull round + one window
        comb = misc + 256;
        // shared scratch: backward combine [kWin][16] / (rays phase) per-wave entry lists
        // [waves][kList][8] / (backward pairs) per-wave pair slots [waves][64][kSlot]
        int ncomb = kWin * 16;
        if ((tb / 64) * kList * 8 > ncomb) ncomb = (tb / 64) * kList * 8;
        if (bwd && (tb / 64) * 64 * kSlot > ncomb) ncomb = (tb / 64) * 64 * kSlot;
        total = comb + ncomb;
    }
};

__device__ __forceinline__ float quadric(const float* M, float dx, float dy, float dz) {
    const float t0 = fmaf(M[0], dx, fmaf(M[1], dy, M[2] * dz));
    const float t1 = fmaf(M[3], dy, M[4] * dz);
    return fmaf(dx, t0, fmaf(dy, t1, dz * dz * M[5]));
}

// 1 - exp(-x) for 0 <= x <= 1/64 (x = sigma pdf c dT <= c dT): x (1 - x/2 + x^2/6 - x^3/24), truncation
// x^4/120 <= 5e-10 relative.  Used instead of an exp (and of its cancelling 1 - exp) when c dT <= 1/64
// (C3: c dT = 1.25e-3), which makes the whole launch take the polynomial (a kernel-uniform branch).
constexpr float kSmallX = 1.0f / 64.0f;
__device__ __forceinline__ float om_exp_small(float x) {
    return x * fmaf(x, fmaf(x, fmaf(x, -1.0f / 24.0f, 1.0f / 6.0f), -0.5f), 1.0f);
}

// value of lane s (wave-uniform s) as a scalar
__device__ __forceinline__ float rlf(float v, int s) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), s));
}
__device__ __forceinline__ int rli(int v, int s) { return __builtin_amdgcn_readlane(v, s); }

// SH albedo term sh = f . Y(dir) over the active coefficients
__device__ __forceinline__ float sh_dot(const float* f, const float* Y, int K) {
    float sh = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxK; ++c)
        if (c < K) sh += f[c] * Y[c];
    return sh;
}

__device__ __forceinline__ float wave_incl_sum(float x) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float u = __shfl_up(x, off);
        if (lane >= off) x += u;
    }
    return x;
}

__device__ __forceinline__ float wave_incl_suffix(float x) {
    const int lane = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float u = __shfl_down(x, off);
        if (lane + off < 64) x += u;
    }
    return x;
}

__device__ __forceinline__ int wave_min_i(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = min(x, __shfl_xor(x, off));
    return x;
}

__device__ __forceinline__ int wave_max_i(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = max(x, __shfl_xor(x, off));
    return x;
}

// slab test of the half-infinite ray o + t d against a box (cuda_utils.cuh:97-121, IEEE ops)
__device__ __forceinline__ bool slab_hit(const float* bb, float ox, float oy, float oz, float ix, float iy, float iz) {
    const float tx0 = (bb[0] - ox) * ix, tx1 = (bb[3] - ox) * ix;
    const float ty0 = (bb[1] - oy) * iy, ty1 = (bb[4] - oy) * iy;
    const float tz0 = (bb[2] - oz) * iz, tz1 = (bb[5] - oz) * iz;
    const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
    const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return tmax >= tmin && tmax >= 0.0f;
}

// per-Gaussian cull record: mu and the radius of a sphere containing the support / the box
template <int SEL>
__global__ __launch_bounds__(256) void cull_prep_kernel(nlosgr_gaussians g, const GaussRec* recs, float mc,
                                                        float4* cull, float* bbox) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.ng) return;
    const GaussRec r = recs[i];
    float rad;
    if (SEL == NLOSGR_SELECT_AABB) {
        float b[6];
        gauss_bbox<NLOSGR_PRESET_CUDA>(g, i, 3.0f, b);
        for (int t = 0; t < 6; ++t) bbox[6 * (size_t)i + t] = b[t];
        const float ex = 0.5f * (b[3] - b[0]), ey = 0.5f * (b[4] - b[1]), ez = 0.5f * (b[5] - b[2]);
        const float cx = 0.5f * (b[3] + b[0]), cy = 0.5f * (b[4] + b[1]), cz = 0.5f * (b[5] + b[2]);
        // sphere around mu holding the whole box (the box is centred on mu up to rounding)
        const float off = sqrtf((cx - r.a.x) * (cx - r.a.x) + (cy - r.a.y) * (cy - r.a.y) + (cz - r.a.z) * (cz - r.a.z));
        rad = (sqrtf(ex * ex + ey * ey + ez * ez) + off) * 1.0001f + 1e-7f;
    } else {
        rad = mc > 0.f ? mc * r.d.y * 1.0001f + 1e-7f : INFINITY;
    }
    cull[i] = make_float4(r.a.x, r.a.y, r.a.z, rad);
}

// Tile cull test: the sphere (c.xyz, radius c.w) against the tile's cone (axis a, half-angle h):
// angle(v, a) <= h + asin(R / |v|)  <=>  v.a >= cos h sqrt(|v|^2 - R^2) - sin h R, v = mu - p.  No fp
// contraction (explicit fmaf), so tile_bin_kernel and the in-kernel cull agree bit for bit.
__device__ __forceinline__ bool cone_hit(float4 c, float px, float py, float pz, float ax, float ay, float az, float ch,
                                         float shh, bool pass_all) {
#pragma clang fp contract(off)
    const float vx = c.x - px, vy = c.y - py, vz = c.z - pz;
    const float d2 = fmaf(vz, vz, fmaf(vy, vy, vx * vx));
    const float R2 = c.w * c.w;
    if (pass_all || d2 <= R2 || !(c.w < INFINITY)) return true;
    return fmaf(vz, az, fmaf(vy, ay, vx * ax)) >= fmaf(ch, sqrtf(d2 - R2), -(shh * c.w));
}

// Tile cones of one launch's items (wave = (wall point, tile), lane = ray of the tile): the mean ray
// direction as axis, the largest ray angle to it + 2e-4 as half-angle (pass-all past 1.5 rad).
// cones[(p * ntiles + t) * 8] = (ax, ay, az, cos h, sin h, pass_all, 0, 0).
__global__ __launch_bounds__(256) void tile_cone_kernel(nlosgr_geometry geo, int ti, int tj, int ntile_j, int ntiles,
                                                        float* cones) {
    const long long item = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (item >= (long long)geo.nwall * ntiles) return;
    const int lane = lane_id();
    const int p = (int)(item / ntiles), t = (int)(item - (long long)p * ntiles);
    const int nt = geo.nt, np_ = geo.np, rt = ti * tj;
    const int ti0 = (t / ntile_j) * ti, tj0 = (t % ntile_j) * tj;
    const int i = ti0 + lane / tj, j = tj0 + lane % tj;
    const bool v = lane < rt && i < nt && j < np_;
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (v) {
        const float st = geo.sin_theta[(size_t)p * nt + i];
        dx = st * geo.cos_phi[(size_t)p * np_ + j];
        dy = st * geo.sin_phi[(size_t)p * np_ + j];
        dz = geo.cos_theta[(size_t)p * nt + i];
    }
    float sx = dx, sy = dy, sz = dz;
    for (int off = 32; off > 0; off >>= 1) {
        sx += __shfl_xor(sx, off); sy += __shfl_xor(sy, off); sz += __shfl_xor(sz, off);
    }
    const float n = sqrtf(sx * sx + sy * sy + sz * sz);
    const float ax = n > 0.f ? sx / n : 0.f, ay = n > 0.f ? sy / n : 0.f, az = n > 0.f ? sz / n : 1.f;
    float c = v ? fminf(1.0f, dx * ax + dy * ay + dz * az) : 1.0f;
    for (int off = 32; off > 0; off >>= 1) c = fminf(c, __shfl_xor(c, off));
    const float h = acosf(c) + 2e-4f;
    if (lane == 0) {
        float* o = cones + item * 8;
        *reinterpret_cast<float4*>(o) = make_float4(ax, ay, az, cosf(h));
        *reinterpret_cast<float4*>(o + 4) = make_float4(sinf(h), (h > 1.5f || n == 0.f) ? 1.f : 0.f, 0.f, 0.f);
    }
}

// Tile binning (north_star's "tile binning"): for each wall point of the launch and each tile, one bit per
// Gaussian: does its cull sphere pass the tile's cone (cone_hit, the in-kernel cull's test).  Workgroup =
// (1024-Gaussian chunk, wall point), thread = Gaussian; per tile the wave's ballot is one 64-Gaussian word,
// staged in LDS so each tile's 16 words of the chunk go out as one 128-B store.  Rows [p][t][nwords] keep
// index order, so the tile kernel's queue (and path C's first-256-by-index rule) sees exactly the culled
// sequence it would have built itself, without testing every Gaussian for every item.
constexpr int kBinTB = 1024;
__global__ __launch_bounds__(kBinTB) void tile_bin_kernel(const float4* __restrict__ cull, int ng, nlosgr_geometry geo,
                                                          int ntiles, int nwords, const float* __restrict__ cones,
                                                          unsigned long long* masks) {
    __shared__ float cs[64 * 8];
    __shared__ unsigned long long wb[64][kBinTB / 64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
    const int p = blockIdx.y;
    const int g = blockIdx.x * kBinTB + tid;
    const float4 c = g < ng ? cull[g] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float px = geo.wall[3 * p], py = geo.wall[3 * p + 1], pz = geo.wall[3 * p + 2];
    const float* cp = cones + (size_t)p * ntiles * 8;
    for (int tb = 0; tb < ntiles; tb += 64) {
        const int nb = min(64, ntiles - tb);
        __syncthreads();
        if (tid < nb * 8) cs[tid] = cp[(size_t)tb * 8 + tid];
        __syncthreads();
        for (int tt = 0; tt < nb; ++tt) {
            const float* q = cs + tt * 8;
            const bool hit = g < ng && cone_hit(c, px, py, pz, q[0], q[1], q[2], q[3], q[4], q[5] != 0.f);
            const unsigned long long w = __builtin_amdgcn_ballot_w64(hit);
            if (lane == 0) wb[tt][wave] = w;
        }
        __syncthreads();
        const int tt = tid / (kBinTB / 64), wv = tid % (kBinTB / 64);
        const int word = blockIdx.x * (kBinTB / 64) + wv;
        if (tt < nb && word < nwords) masks[((size_t)p * ntiles + tb + tt) * nwords + word] = wb[tt][wv];
    }
}

// ------------------------------------------------------------------------------------------
// the tile kernel (forward: BWD = false; backward: BWD = true)
// ------------------------------------------------------------------------------------------
template <int SEL, bool DENSE, bool OCCL, bool BWD>
__global__ __launch_bounds__(tile_threads<BWD>()) void tile_kernel(TArgs k) {
    constexpr int kTB = tile_threads<BWD>();
    constexpr int kTW = kTB / 64;
    extern __shared__ __align__(16) float sm[];
    const int nr = k.geo.nr, nt = k.geo.nt, np_ = k.geo.np;
    const TLayout L(k.rt, nr, kTB, BWD);
    float2* rows = reinterpret_cast<float2*>(sm + L.rows);
    float* stage = sm + L.stage;
    int* queue = reinterpret_cast<int*>(sm + L.queue);
    float* comb = sm + L.comb;
    float* misc = sm + L.misc;
    int* icnt = reinterpret_cast<int*>(misc);          // [64] AABB cap counters per ray
    int* ihalf = icnt + 64;                             // [64] per-window hits of the first staged half
    constexpr int kCullU = cull_u<BWD>();
    int* iwave = icnt + 128;                            // [kCullU][kTW] cull counts per wave / bin-round scan (64 ints)
    static_assert(cull_u<BWD>() * kTW <= 64 && 3 * kTW <= 64, "per-wave cull counts overflow misc[128, 192)");
    const int tid = threadIdx.x, wave = tid >> 6, lane = lane_id();
    const int RT = k.rt;
    // AABB selection: each selected Gaussian over the samples within the cutoff (5.7 sigma = parity
    // grade: terms below 9e-8 of its peak dropped), or the whole representable ray (cutoff <= 0)
    const float mc2 = SEL == NLOSGR_SELECT_AABB ? (k.opt.cutoff > 0.f ? k.opt.cutoff * k.opt.cutoff : kFullM2)
                                                : k.opt.cutoff * k.opt.cutoff;
    const float r0 = k.geo.r[0];
    const float dr = nr > 1 ? (k.geo.r[nr - 1] - r0) / (float)(nr - 1) : 1.0f;
    const float inv_dr = 1.0f / dr;
    const float cdt = k.opt.c_deltaT;
    const float ncdt = -cdt * kLog2e;   // exp(-x c dT) = exp2(x ncdt)
    const bool small_x = cdt <= kSmallX;  // 1 - exp(-sigma pdf c dT) by om_exp_small
    // backward pair walks with sigma folded out and the quartic 1 - exp(-x) (kernel-uniform): walks bounded by a
    // cutoff <= 6 sigma (for the recurrence variant: the ratio exp2(ga (2t + 1)) stays below 2^47 inside the
    // support), and with occlusion only at c dT <= 1/64
    const bool walk_rec = NLOSGR_WALK_REC && !DENSE && k.opt.cutoff > 0.f && mc2 <= 36.f && (!OCCL || small_x);
    const int nch = (nr + 63) / 64;
    const int deg = k.g.sh_degree, K = (deg + 1) * (deg + 1);

    unsigned long long tc = 0, tcull = 0, tstage = 0, trays = 0, tscan = 0, nwin = 0, nent = 0, nec = 0, nchk = 0;
#define TDIAG(acc)                                   \
    if (kDiag && k.diag && tid == 0) {               \
        const unsigned long long t1 = clock64();     \
        acc += t1 - tc;                              \
        tc = t1;                                     \
    }
    if (kDiag && k.diag && tid == 0) tc = clock64();
    __shared__ long long s_next;
    // forward: a slot takes the next unclaimed item when it finishes one (per-item outputs, so the
    // order does not matter); backward: items s, s + nslot, ... (fixed order of the slot's sums)
    auto advance = [&](long long it) -> long long {
        if (BWD || !k.next) return it + k.nslot;
        __syncthreads();
        if (tid == 0) s_next = (long long)k.nslot + (long long)atomicAdd(k.next, 1ull);
        __syncthreads();
        return s_next;
    };
    for (long long item = blockIdx.x; item < k.nitems; item = advance(item)) {
        // item -> (wall point, tile), the tile index rotated by the wall point: with nslot a multiple of
        // ntiles a slot's static items would otherwise all sit at one tile position of the angular grid
        // (C3: slot s always tile s % 64, so the slots holding central tiles set the launch time)
        const int p = (int)(item / k.ntiles);
        const int t = (int)((item - (long long)p * k.ntiles + p + k.pbase) % k.ntiles);
        const int ti0 = (t / k.ntile_j) * k.ti, tj0 = (t % k.ntile_j) * k.tj;
        const float px = k.geo.wall[3 * p], py = k.geo.wall[3 * p + 1], pz = k.geo.wall[3 * p + 2];
        const float* sth = k.geo.sin_theta + (size_t)p * nt;
        const float* cth = k.geo.cos_theta + (size_t)p * nt;
        const float* sph = k.geo.sin_phi + (size_t)p * np_;
        const float* cph = k.geo.cos_phi + (size_t)p * np_;
        __syncthreads();   // previous item done with LDS
        if (tid < 64) icnt[tid] = 0;
        for (int x = tid; x < RT * nr; x += kTB) rows[x] = make_float2(0.f, 0.f);
        __syncthreads();
        // the tile's cone from the table (tile_cone_kernel: the same values the bins were built with)
        const float* cn = k.cones + ((size_t)p * k.ntiles + t) * 8;
        const float4 cA = *reinterpret_cast<const float4*>(cn), cB = *reinterpret_cast<const float4*>(cn + 4);
        const float ax = cA.x, ay = cA.y, az = cA.z, ch = cA.w, shh = cB.x;
        const bool pass_all = cB.y != 0.f;
        // tile bins: this item's row of 64-Gaussian hit words (index order)
        const unsigned long long* mrow = k.masks ? k.masks + ((size_t)p * k.ntiles + t) * k.nwords : nullptr;

        // ---------------- sweeps over the Gaussians (forward: 1; backward: 2) ----------------
        for (int sweep = 0; sweep < (BWD ? 2 : 1); ++sweep) {
            const bool pairs = BWD && sweep == 1;
            if (pairs) {
                // the scan turned the rows into (a, b); reset the cap counters for the replay
                if (tid < 64) icnt[tid] = 0;
                __syncthreads();
            }
            // backward, first sweep: without occlusion the scan needs no (D, W) rows at all; with the
            // row cache they are the forward's, reloaded (coalesced) instead of recomputed
            const bool skip0 = BWD && !pairs && (!OCCL || k.rcache != nullptr);
            if (BWD && !pairs && OCCL && k.rcache) {
                const float2* src = k.rcache + (size_t)item * RT * nr;
                for (int x = tid; x < RT * nr; x += kTB) rows[x] = src[x];
                __syncthreads();
            }
            int qn = 0, qh = 0;   // live queue entries: [qh, qn)
            bool capped = false;   // AABB: every ray of the tile holds its 256 selections (nothing later counts)
            // the cull records of the next round are loaded one round ahead (their L2 round trip overlaps
            // the current round's barriers and windows); kCullU blocks of kTB Gaussians per round
            float4 cnext[kCullU];
#pragma unroll
            for (int u = 0; u < kCullU; ++u) {
                cnext[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (!skip0 && !mrow && u * kTB + tid < k.g.ng) cnext[u] = k.cull[u * kTB + tid];
            }
            // g0: the next Gaussian (in-kernel cull) or the next 64-Gaussian word of the item's bin row
            const int gend = mrow ? k.nwords : k.g.ng;
            for (int g0 = 0; !skip0 && !capped && (g0 < gend || qn > qh);) {
                if (g0 < gend) {
                    if (qh > 0) {
                        // what the windows left (< kWin entries) moves to the front once per cull round
                        const int rest = qn - qh;
                        int keep = 0;
                        if (tid < rest) keep = queue[qh + tid];
                        __syncthreads();
                        if (tid < rest) queue[tid] = keep;
                        qn = rest;
                        qh = 0;
                    }
                    if (mrow) {
                        // ---- bin round: thread = one 64-Gaussian word; the words whose hits fit the queue
                        // (kCullU x kTB entries; a prefix of the threads) append their indices in order ----
                        constexpr int cap = kCullU * kTB;
                        const int wi = g0 + tid;
                        const unsigned long long wd = wi < gend ? mrow[wi] : 0ull;
                        const int h = __popcll(wd);
                        int incl = h;
#pragma unroll
                        for (int off = 1; off < 64; off <<= 1) {
                            const int u = __shfl_up(incl, off);
                            if (lane >= off) incl += u;
                        }
                        if (lane == 63) iwave[wave] = incl;
                        __syncthreads();
                        int base = 0;
#pragma unroll
                        for (int w = 0; w < kTW; ++w) base += w < wave ? iwave[w] : 0;
                        const int ex = base + incl - h;
                        const bool take = wi < gend && ex + h <= cap;
                        if (take) {
                            unsigned long long m = wd;
                            int o = qn + ex;
                            while (m) {
                                queue[o++] = wi * 64 + (int)__builtin_ctzll(m);
                                m &= m - 1ull;
                            }
                        }
                        const int wtake = __popcll(__builtin_amdgcn_ballot_w64(take));
                        const int went = wave_max_i(take ? ex + h : 0);
                        if (lane == 0) {
                            iwave[kTW + wave] = wtake;
                            iwave[2 * kTW + wave] = went;
                        }
                        __syncthreads();
                        int nw = 0, ne = 0;
#pragma unroll
                        for (int w = 0; w < kTW; ++w) {
                            nw += iwave[kTW + w];
                            ne = max(ne, iwave[2 * kTW + w]);
                        }
                        g0 += nw;
                        qn += ne;
                        __syncthreads();   // (iwave is rewritten by the next round)
                        TDIAG(tcull)
                    } else {
                    bool hit[kCullU];
                    unsigned long long m[kCullU];
#pragma unroll
                    for (int u = 0; u < kCullU; ++u) {
                        const int gi = g0 + u * kTB + tid;
                        const float4 c = cnext[u];
                        if (gi + kCullU * kTB < k.g.ng) cnext[u] = k.cull[gi + kCullU * kTB];
                        hit[u] = gi < k.g.ng && cone_hit(c, px, py, pz, ax, ay, az, ch, shh, pass_all);
                        m[u] = __builtin_amdgcn_ballot_w64(hit[u]);
                        if (lane == 0) iwave[u * kTW + wave] = __popcll(m[u]);
                    }
                    __syncthreads();
                    // the per-wave counts as int4 reads; block u's hits follow all of block u - 1's
                    int run = qn;
                    const int4* iw4 = reinterpret_cast<const int4*>(iwave);
#pragma unroll
                    for (int u = 0; u < kCullU; ++u) {
                        int base = run, tot = 0;
#pragma unroll
                        for (int w4 = 0; w4 < kTW / 4; ++w4) {
                            const int4 c4 = iw4[u * (kTW / 4) + w4];
                            const int cw[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                            for (int v = 0; v < 4; ++v) {
                                base += 4 * w4 + v < wave ? cw[v] : 0;
                                tot += cw[v];
                            }
                        }
                        if (hit[u]) queue[base + lanes_below(m[u])] = g0 + u * kTB + tid;
                        run += tot;
                    }
                    qn = run;
                    __syncthreads();
                    TDIAG(tcull)
                    g0 += kCullU * kTB;
                    }
                }
                const bool last = g0 >= gend;
                // ---- windows of up to 128 staged Gaussians ----
                while (qn - qh >= kWin || (last && qn > qh)) {
                    const int nst = min(qn - qh, kWin);
                    if (tid < nst) {
                        const int gi = queue[qh + tid];
                        const GaussRec rec = k.recs[gi];
                        // the SH row is loaded with the record (its round trip overlaps the record's)
                        float fr[kMaxK];
#pragma unroll
                        for (int c = 0; c < kMaxK; ++c) fr[c] = c < K ? k.g.features[(size_t)gi * k.g.k_feat + c] : 0.f;
                        float* o = stage + tid * kStage;
                        const float A[9] = {rec.b.x, rec.b.y, rec.b.z, rec.b.w, rec.c.x, rec.c.y, rec.c.z, rec.c.w, rec.d.x};
                        const float q0 = px - rec.a.x, q1 = py - rec.a.y, q2 = pz - rec.a.z;
                        float u0[3];
                        for (int r = 0; r < 3; ++r) u0[r] = A[3 * r] * q0 + A[3 * r + 1] * q1 + A[3 * r + 2] * q2;
                        for (int x = 0; x < 9; ++x) o[x] = A[x];
                        o[9] = u0[0]; o[10] = u0[1]; o[11] = u0[2];
                        if (SEL == NLOSGR_SELECT_AABB) {
                            for (int x = 0; x < 6; ++x) o[12 + x] = k.bbox[6 * (size_t)gi + x];
                        } else if (!DENSE) {
                            const float N[6] = {rec.d.z, rec.d.w, rec.e.x, rec.e.y, rec.e.z, rec.e.w};
                            const float wv0 = A[0] * u0[0] + A[3] * u0[1] + A[6] * u0[2];
                            const float wv1 = A[1] * u0[0] + A[4] * u0[1] + A[7] * u0[2];
                            const float wv2 = A[2] * u0[0] + A[5] * u0[1] + A[8] * u0[2];
                            const float kap = u0[0] * u0[0] + u0[1] * u0[1] + u0[2] * u0[2] - mc2;
                            o[12] = wv0 * wv0 - kap * N[0];
                            o[13] = 2.0f * (wv0 * wv1 - kap * N[1]);
                            o[14] = 2.0f * (wv0 * wv2 - kap * N[2]);
                            o[15] = wv1 * wv1 - kap * N[3];
                            o[16] = 2.0f * (wv1 * wv2 - kap * N[4]);
                            o[17] = wv2 * wv2 - kap * N[5];
                        }
                        o[18] = rec.a.w;
                        // rho = max(0, 0.5 + SH(dir(mu - p))) (volume_renderer.cu:109-111)
                        float dx, dy, dz, nrm;
                        view_dir<NLOSGR_PRESET_CUDA>(-q0, -q1, -q2, dx, dy, dz, nrm);
                        float Y[kMaxK];
                        sh_basis<NLOSGR_PRESET_CUDA>(deg, dx, dy, dz, Y);
                        const float sh = sh_dot(fr, Y, K);
                        o[19] = fmaxf(sh + 0.5f, 0.0f);
                    }
                    __syncthreads();
                    TDIAG(tstage)
                    ++nwin;
                    if (!pairs) {
                        // ---- rays: wave = ray, lane = staged entry, then lane = bin ----
                        for (int r = wave; r < RT; r += kTW) {
                            const int i = ti0 + r / k.tj, j = tj0 + r % k.tj;
                            if (i >= nt || j >= np_) continue;
                            const float dx = sth[i] * cph[j], dy = sth[i] * sph[j], dz = cth[i];
                            const float ix = 1.0f / (dx + 1e-8f), iy = 1.0f / (dy + 1e-8f), iz = 1.0f / (dz + 1e-8f);
                            for (int e0 = 0; e0 < nst; e0 += 64) {
                                const int e = e0 + lane;
                                const bool valid = e < nst;
                                const float* o = stage + (valid ? e : 0) * kStage;
                                bool sel = valid;
                                if (SEL == NLOSGR_SELECT_AABB) {
                                    sel = valid && slab_hit(o + 12, px, py, pz, ix, iy, iz);
                                    const unsigned long long m = __builtin_amdgcn_ballot_w64(sel);
                                    const int c0 = icnt[r];
                                    sel = sel && c0 + lanes_below(m) < kCap;
                                    wave_sync();
                                    if (lane == 0) icnt[r] = min(kCap, c0 + __popcll(m));
                                    wave_sync();
                                } else if (!DENSE && valid) {
                                    sel = quadric(o + 12, dx, dy, dz) >= 0.f;
                                }
                                float ks = 0.f, ga = 0.f, al = -INFINITY, sg = 0.f, rho = 0.f;
                                int kl = nr, kh = -1;
                                if (sel) {
                                    float v[3];
                                    for (int x = 0; x < 3; ++x) v[x] = o[3 * x] * dx + o[3 * x + 1] * dy + o[3 * x + 2] * dz;
                                    const float a = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
                                    const float b = o[9] * v[0] + o[10] * v[1] + o[11] * v[2];
                                    const float ia = 1.0f / a;
                                    const float ts = -b * ia;
                                    const float z0 = o[9] + ts * v[0], z1 = o[10] + ts * v[1], z2 = o[11] + ts * v[2];
                                    const float m2min = z0 * z0 + z1 * z1 + z2 * z2;
                                    ks = (ts - r0) * inv_dr;
                                    if (DENSE) {
                                        kl = 0; kh = nr - 1;
                                    } else if (m2min <= mc2) {
                                        const float hk = sqrtf((mc2 - m2min) * ia) * inv_dr;
                                        kl = fidx(ceilf(ks - hk), 0, nr);
                                        kh = fidx(floorf(ks + hk), -1, nr - 1);
                                    }
                                    ga = -0.5f * kLog2e * a * dr * dr;
                                    al = -0.5f * kLog2e * m2min;
                                    sg = o[18];
                                    rho = o[19];
                                }
                                const bool live = kl <= kh;
                                const unsigned long long lm = __builtin_amdgcn_ballot_w64(live);
                                if (kDiag && k.diag && tid == 0) nent += __popcll(lm);
                                if (!lm) continue;
                                // live entries (index order) go to this wave's LDS list, kList per pass;
                                // lane = bin then reads them as broadcasts (uniform address)
                                const int lrank = lanes_below(lm);
                                float4* el = reinterpret_cast<float4*>(comb) + wave * kList * 2;
                                for (int pb = 0; pb < __popcll(lm); pb += kList) {
                                    const bool inp = live && lrank >= pb && lrank < pb + kList;
                                    const unsigned long long pm = __builtin_amdgcn_ballot_w64(inp);
                                    wave_sync();
                                    if (inp) {
                                        el[2 * (lrank - pb)] = make_float4(ks, ga, al, sg);
                                        el[2 * (lrank - pb) + 1] =
                                            make_float4(rho, __int_as_float(kl), __int_as_float(kh - kl), 0.f);
                                    }
                                    wave_sync();
                                    const int lo = wave_min_i(inp ? kl : nr);
                                    const int hi = wave_max_i(inp ? kh : -1);
                                    for (int c = lo >> 6; c <= (hi >> 6); ++c) {
                                        unsigned long long cm =
                                            __builtin_amdgcn_ballot_w64(inp && kl <= c * 64 + 63 && kh >= c * 64);
                                        if (kDiag && k.diag && tid == 0) { ++nchk; nec += __popcll(cm); }
                                        if (!cm) continue;
                                        const int kb = c * 64 + lane;
                                        const float kf = (float)kb;
                                        float accD = 0.f, accW = 0.f;
                                        // the entry loop per small-c dT form (a kernel-uniform flag: one scalar branch per
                                        // chunk instead of both forms per entry; C3 occl AABB forward 1341 -> 1260 ms)
                                        auto entries = [&](auto smallc) {
                                            constexpr bool kSmall = decltype(smallc)::value;
                                            while (cm) {
                                                const int s = __builtin_ctzll(cm);
                                                cm &= cm - 1;
                                                const int idx = __popcll(pm & ((1ull << s) - 1ull));
                                                const float4 e0 = el[2 * idx], e1 = el[2 * idx + 1];
                                                const int skl = __float_as_int(e1.y), slen = __float_as_int(e1.z);   // kh - kl
                                                const float tt = kf - e0.x;
                                                const float pdf = fast_exp2(fmaf(e0.y, tt * tt, e0.z));
                                                // kl <= kb <= kh as one unsigned range compare
                                                const float cv = (unsigned)(kb - skl) <= (unsigned)slen ? e0.w * pdf : 0.f;
                                                if (OCCL) {
                                                    accD += cv;
                                                    // (small x: the cubic x (1 - x/2 + x^2/6), x^4/24 <= 1.6e-7 relative at 1/64)
                                                    float w;
                                                    if (kSmall) {
                                                        const float x = cv * cdt;
                                                        w = NLOSGR_TILE_OM3 ? x * fmaf(x, fmaf(x, 1.0f / 6.0f, -0.5f), 1.0f) : om_exp_small(x);
                                                    } else {
                                                        w = 1.0f - fast_exp2(cv * ncdt);
                                                    }
                                                    accW = fmaf(e1.x, w, accW);
                                                } else {
                                                    accW = fmaf(e1.x, cv, accW);
                                                }
                                            }
                                        };
                                        if (small_x) entries(std::integral_constant<bool, true>{});
                                        else entries(std::integral_constant<bool, false>{});
                                        if (kb < nr) {
                                            float2 v = rows[r * nr + kb];
                                            v.x += accD;
                                            v.y += accW;
                                            rows[r * nr + kb] = v;
                                        }
                                    }
                                }
                            }
                        }
                    } else {
                        // ---- pairs (backward): lane = (staged entry, ray group) ----
                        const int half = wave & 1, rg = wave >> 1;
                        const int e = half * 64 + lane;
                        const bool valid = e < nst;
                        const float* o = stage + (valid ? e : 0) * kStage;
                        float A[9], u0[3], sel6[6];
                        for (int x = 0; x < 9; ++x) A[x] = o[x];
                        for (int x = 0; x < 3; ++x) u0[x] = o[9 + x];
                        for (int x = 0; x < 6; ++x) sel6[x] = o[12 + x];
                        const float sg = o[18], rho = o[19];
                        if (SEL == NLOSGR_SELECT_AABB) {
                            // hits of the first staged half per ray (the second half's cap ranks follow them)
                            if (half == 0)
                                for (int r = rg; r < RT; r += 4) {
                                    const int i = ti0 + r / k.tj, j = tj0 + r % k.tj;
                                    bool h = false;
                                    if (valid && i < nt && j < np_) {
                                        const float dx = sth[i] * cph[j], dy = sth[i] * sph[j], dz = cth[i];
                                        h = slab_hit(sel6, px, py, pz, 1.0f / (dx + 1e-8f), 1.0f / (dy + 1e-8f),
                                                     1.0f / (dz + 1e-8f));
                                    }
                                    const unsigned long long m = __builtin_amdgcn_ballot_w64(h);
                                    if (lane == 0) ihalf[r] = __popcll(m);
                                }
                            __syncthreads();
                        }
                        float dA[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                        float gU[3] = {0.f, 0.f, 0.f};
                        float dsig = 0.f, drho = 0.f;
                        // rays r = rg + 4 (4 rb + kk): blocks of four per ray group
                        for (int rb = 0; 16 * rb < RT; ++rb) {
                        // (1) lane = entry: which of the block's 4 rays select the entry and cross its
                        //     support -> one live mask per ray
                        unsigned long long live_m[4];
                        int cls[4] = {0, 0, 0, 0};         // (support selection) walk-length class
                        float rdx[4], rdy[4], rdz[4];   // ray directions (wave-uniform)
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) {
                            live_m[kk] = 0ull;
                            rdx[kk] = rdy[kk] = rdz[kk] = 0.f;
                            const int r = rg + 4 * (4 * rb + kk);
                            if (r >= RT) continue;
                            const int i = ti0 + r / k.tj, j = tj0 + r % k.tj;
                            if (i >= nt || j >= np_) continue;
                            const float dx = sth[i] * cph[j], dy = sth[i] * sph[j], dz = cth[i];
                            rdx[kk] = dx; rdy[kk] = dy; rdz[kk] = dz;
                            bool sel = valid;
                            if (SEL == NLOSGR_SELECT_AABB) {
                                sel = valid && slab_hit(sel6, px, py, pz, 1.0f / (dx + 1e-8f), 1.0f / (dy + 1e-8f),
                                                        1.0f / (dz + 1e-8f));
                                const unsigned long long m = __builtin_amdgcn_ballot_w64(sel);
                                const int rank = icnt[r] + (half ? ihalf[r] : 0) + lanes_below(m);
                                sel = sel && rank < kCap;
                            } else if (!DENSE && valid) {
                                sel = quadric(sel6, dx, dy, dz) >= 0.f;
                            }
                            bool live = false;
                            if (sel) {
                                float v[3];
                                for (int x = 0; x < 3; ++x) v[x] = A[3 * x] * dx + A[3 * x + 1] * dy + A[3 * x + 2] * dz;
                                const float a = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
                                const float b = u0[0] * v[0] + u0[1] * v[1] + u0[2] * v[2];
                                const float ia = 1.0f / a;
                                const float ts = -b * ia;
                                const float z0 = u0[0] + ts * v[0], z1 = u0[1] + ts * v[1], z2 = u0[2] + ts * v[2];
                                const float m2min = z0 * z0 + z1 * z1 + z2 * z2;
                                if (DENSE) {
                                    live = true;
                                } else if (m2min <= mc2) {
                                    const float ks = (ts - r0) * inv_dr;
                                    const float hk = sqrtf((mc2 - m2min) * ia) * inv_dr;
                                    if constexpr (SEL == NLOSGR_SELECT_SUPPORT) {
                                        const int klo = fidx(ceilf(ks - hk), 0, nr), khi = fidx(floorf(ks + hk), -1, nr - 1);
                                        live = klo <= khi;
                                        const int len = khi - klo + 1;
                                        cls[kk] = len >= kWalkC0 ? 0 : (len >= kWalkC1 ? 1 : (len >= kWalkC2 ? 2 : 3));
                                    } else {
                                        live = fidx(ceilf(ks - hk), 0, nr) <= fidx(floorf(ks + hk), -1, nr - 1);
                                    }
                                }
                            }
                            live_m[kk] = __builtin_amdgcn_ballot_w64(live);
                        }
                        // support selection: this lane's pairs' places in the length-sorted pass order
                        int pos[4] = {-1, -1, -1, -1};
                        int nsort = 0;
                        if constexpr (SEL == NLOSGR_SELECT_SUPPORT) {
                            int np0 = 0;
#pragma unroll
                            for (int kk = 0; kk < 4; ++kk) np0 += __popcll(live_m[kk]);
                            if (np0 > 64) {
#pragma unroll
                                for (int c = 0; c < 4; ++c)
#pragma unroll
                                    for (int kk = 0; kk < 4; ++kk) {
                                        const bool mine = ((live_m[kk] >> lane) & 1ull) && cls[kk] == c;
                                        const unsigned long long m = __builtin_amdgcn_ballot_w64(mine);
                                        if (mine) pos[kk] = nsort + lanes_below(m);
                                        nsort += __popcll(m);
                                    }
                            }
                        }
                        int lbase[5];
                        lbase[0] = 0;
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) lbase[kk + 1] = lbase[kk] + __popcll(live_m[kk]);
                        float* slots = comb + wave * 64 * kSlot;
                        // (2) the live (entry, ray) pairs, 64 per pass, one per lane: lane = pair walks
                        //     the pair's in-support bins and leaves its moments in the wave's slots;
                        // (3) lane = entry folds its pairs in ray order (fixed order: deterministic)
                        for (int pb = 0; pb < lbase[4]; pb += 64) {
                            wave_sync();
#pragma unroll
                            for (int kk = 0; kk < 4; ++kk) {
                                const int idx = (nsort ? pos[kk] : lbase[kk] + lanes_below(live_m[kk])) - pb;
                                if (((live_m[kk] >> lane) & 1ull) && idx >= 0 && idx < 64)
                                    slots[idx * kSlot + 5] = __int_as_float((kk << 8) | lane);
                            }
                            wave_sync();
                            if (pb + lane < lbase[4]) {
                                const int key = __float_as_int(slots[lane * kSlot + 5]);
                                const int kk = key >> 8, ew = half * 64 + (key & 255);
                                const float dx = kk == 0 ? rdx[0] : kk == 1 ? rdx[1] : kk == 2 ? rdx[2] : rdx[3];
                                const float dy = kk == 0 ? rdy[0] : kk == 1 ? rdy[1] : kk == 2 ? rdy[2] : rdy[3];
                                const float dz = kk == 0 ? rdz[0] : kk == 1 ? rdz[1] : kk == 2 ? rdz[2] : rdz[3];
                                const float* ow = stage + ew * kStage;
                                float v[3];
                                for (int x = 0; x < 3; ++x) v[x] = ow[3 * x] * dx + ow[3 * x + 1] * dy + ow[3 * x + 2] * dz;
                                const float wu0 = ow[9], wu1 = ow[10], wu2 = ow[11], wsg = ow[18], wrho = ow[19];
                                const float a = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
                                const float b = wu0 * v[0] + wu1 * v[1] + wu2 * v[2];
                                const float ia = 1.0f / a;
                                const float ts = -b * ia;
                                const float z0 = wu0 + ts * v[0], z1 = wu1 + ts * v[1], z2 = wu2 + ts * v[2];
                                const float m2min = z0 * z0 + z1 * z1 + z2 * z2;
                                const float ks = (ts - r0) * inv_dr;
                                int kl = 0, kh = nr - 1;
                                if (!DENSE) {
                                    const float hk = sqrtf(fmaxf(mc2 - m2min, 0.f) * ia) * inv_dr;
                                    kl = fidx(ceilf(ks - hk), 0, nr);
                                    kh = fidx(floorf(ks + hk), -1, nr - 1);
                                }
                                const float ga = -0.5f * kLog2e * a * dr * dr;
                                const float al = -0.5f * kLog2e * m2min;
                                float m0 = 0.f, m1 = 0.f, m2 = 0.f, ps = 0.f, pr = 0.f;
                                const float2* row = rows + (rg + 4 * (4 * rb + kk)) * nr;
                                const float rc = wrho * cdt;
                                float tt = (float)kl - ks;   // bin offset from the closest approach, stepped by 1
                                // the rows are read-only here: reads run two bins ahead of their use (past the
                                // segment end they stay inside the LDS allocation and are not used)
                                float2 ab0 = row[kl], ab1 = row[kl + 1];
                                if (walk_rec) {
                                    // sigma folded out of the loop (G = dc pdf, ps = sum dc pdf = m0 before the sigma
                                    // scaling); occlusion at c dT <= 1/64: 1 - exp(-x), x = sigma c dT pdf, as a
                                    // cubic in pdf
                                    const float kx = wsg * cdt;
                                    // cubic: the x^4 / 24 term is <= x^3 / 24 <= 1.6e-7 relative at x = 1/64 (C3: 8e-11)
                                    const float e1 = kx, e2 = -0.5f * kx * kx, e3 = kx * kx * kx * (1.0f / 6.0f);
                                    auto omf = [e1, e2, e3](float pv) { return pv * fmaf(pv, fmaf(pv, e3, e2), e1); };
                                    auto bin = [&](float pdf, float2 ab, float t) {
                                        float dc;
                                        if (OCCL) {
                                            const float om = omf(pdf);
                                            const float u = ab.x * rc;
                                            dc = fmaf(-u, om, u + ab.y);   // a rho c dT (1 - om) + b
                                            pr = fmaf(ab.x, om, pr);
                                        } else {
                                            dc = ab.x * wrho;
                                            pr = fmaf(ab.x, pdf, pr);      // x sigma below
                                        }
                                        const float G = dc * pdf;
                                        m0 += G;
                                        m1 = fmaf(G, t, m1);
                                        m2 = fmaf(G * t, t, m2);
                                    };
                                    if (kWalkReseed > 0 && OCCL) {   // (AABB without occlusion: 1591 -> 1674 ms with it)
                                        // pdf by the exp2 recurrence (pdf(t + 1) = pdf(t) q, q(t + 1) = q(t) 2^(2 ga)),
                                        // re-seeded with exact exp2 every kWalkReseed bins of the walk: every lane
                                        // starts its walk together, so the re-seed is uniform across the wave
                                        // (round 5's re-seed at absolute bin multiples made some lane re-seed
                                        // almost every step).  Inside the support at m_c^2 <= 36 the ratio's
                                        // exponent stays below 27 (no overflow); error <= kWalkReseed^2 / 4 ulp
                                        const float cc = fast_exp2(2.f * ga);
                                        float pc = 0.f, qc = 0.f;
                                        int it = 0;
#pragma unroll NLOSGR_WALK_UNROLL
                                        for (int kb = kl; kb <= kh; ++kb, tt += 1.f, ++it) {
                                            if ((it & (kWalkReseed - 1)) == 0) {
                                                pc = fast_exp2(fmaf(ga, tt * tt, al));
                                                qc = fast_exp2(ga * fmaf(2.f, tt, 1.f));
                                            }
                                            const float pdf = pc;
                                            pc *= qc;
                                            qc *= cc;
                                            const float2 ab = ab0;
                                            ab0 = ab1;
                                            ab1 = row[kb + 2];
                                            bin(pdf, ab, tt);
                                        }
                                    } else {
#pragma unroll NLOSGR_WALK_UNROLL
                                    for (int kb = kl; kb <= kh; ++kb, tt += 1.f) {
                                        const float pdf = fast_exp2(fmaf(ga, tt * tt, al));
                                        const float2 ab = ab0;
                                        ab0 = ab1;
                                        ab1 = row[kb + 2];
                                        bin(pdf, ab, tt);
                                    }
                                    }
                                    ps = m0;
                                    m0 *= wsg;
                                    m1 *= wsg;
                                    m2 *= wsg;
                                    if (!OCCL) pr *= wsg;
                                } else
#pragma unroll NLOSGR_WALK_UNROLL
                                for (int kb = kl; kb <= kh; ++kb, tt += 1.f) {
                                    const float pdf = fast_exp2(fmaf(ga, tt * tt, al));
                                    const float cv = wsg * pdf;
                                    const float2 ab = ab0;
                                    ab0 = ab1;
                                    ab1 = row[kb + 2];
                                    float dc;
                                    if (OCCL) {
                                        const float om = small_x ? om_exp_small(cv * cdt) : 1.0f - fast_exp2(cv * ncdt);
                                        const float ex = 1.0f - om;
                                        dc = fmaf(ab.x * rc, ex, ab.y);
                                        pr = fmaf(ab.x, om, pr);
                                    } else {
                                        dc = ab.x * wrho;
                                        pr = fmaf(ab.x, cv, pr);
                                    }
                                    ps = fmaf(dc, pdf, ps);
                                    const float G = dc * cv;
                                    m0 += G;
                                    m1 = fmaf(G, tt, m1);
                                    m2 = fmaf(G * tt, tt, m2);
                                }
                                float* sl = slots + lane * kSlot;
                                sl[0] = m0; sl[1] = m1; sl[2] = m2; sl[3] = ps; sl[4] = pr;
                            }
                            wave_sync();
#pragma unroll
                            for (int kk = 0; kk < 4; ++kk) {
                                const int idx = (nsort ? pos[kk] : lbase[kk] + lanes_below(live_m[kk])) - pb;
                                if (!(((live_m[kk] >> lane) & 1ull) && idx >= 0 && idx < 64)) continue;
                                const float* sl = slots + idx * kSlot;
                                const float dx = rdx[kk], dy = rdy[kk], dz = rdz[kk];
                                float v[3];
                                for (int x = 0; x < 3; ++x) v[x] = A[3 * x] * dx + A[3 * x + 1] * dy + A[3 * x + 2] * dz;
                                const float a = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
                                const float b = u0[0] * v[0] + u0[1] * v[1] + u0[2] * v[2];
                                const float ts = -b * (1.0f / a);
                                const float zs[3] = {u0[0] + ts * v[0], u0[1] + ts * v[1], u0[2] + ts * v[2]};
                                dsig += sl[3];
                                drho += sl[4];
                                // pdf = exp(-|z|^2 / 2), z_k = zs + tau_k v, tau = (k - ks) dr:
                                // dL/du0 = -(zs M0 + v M1), dL/dv = -(zs (M1 + ts M0) + v (M2 + ts M1))
                                const float M0 = sl[0], M1 = sl[1] * dr, M2 = sl[2] * dr * dr;
                                const float d3[3] = {dx, dy, dz};
                                for (int x = 0; x < 3; ++x) {
                                    const float gu = -(zs[x] * M0 + v[x] * M1);
                                    const float gv = -(zs[x] * (M1 + ts * M0) + v[x] * (M2 + ts * M1));
                                    gU[x] += gu;
                                    for (int c = 0; c < 3; ++c) dA[3 * x + c] = fmaf(gv, d3[c], dA[3 * x + c]);
                                }
                            }
                        }
                        }
                        // combine the four ray groups per entry in order rg = 0..3 (comb overlaps the
                        // pair slots: every wave must be done with them first)
                        __syncthreads();
                        for (int step = 0; step < 4; ++step) {
                            if (rg == step && valid) {
                                float* cb = comb + e * 16;
                                if (step == 0) {
                                    for (int x = 0; x < 9; ++x) cb[x] = dA[x];
                                    cb[9] = gU[0]; cb[10] = gU[1]; cb[11] = gU[2]; cb[12] = dsig; cb[13] = drho;
                                } else {
                                    for (int x = 0; x < 9; ++x) cb[x] += dA[x];
                                    cb[9] += gU[0]; cb[10] += gU[1]; cb[11] += gU[2]; cb[12] += dsig; cb[13] += drho;
                                }
                            }
                            __syncthreads();
                        }
                        // one record per entry -> the slot's accumulator row (waves 0-1, lane = entry)
                        if (wave < 2 && valid) {
                            const float* cb = comb + e * 16;
                            bool any = false;
                            for (int x = 0; x < 14; ++x) any |= cb[x] != 0.f;
                            if (any) {
                                const int gi = queue[qh + e];
                                // the slot row, the Gaussian's mean and its SH row are loaded up front so the
                                // three memory round trips overlap (the row was read after the compute)
                                float4* dst = reinterpret_cast<float4*>(k.acc + ((size_t)blockIdx.x * k.g.ng + gi) * kRec);
                                float4 acc4[kRec / 4];
#pragma unroll
                                for (int x = 0; x < kRec / 4; ++x) acc4[x] = dst[x];
                                const float4 mu4 = k.recs[gi].a;
                                float fr[kMaxK];
#pragma unroll
                                for (int c = 0; c < kMaxK; ++c) fr[c] = c < K ? k.g.features[(size_t)gi * k.g.k_feat + c] : 0.f;
                                const float q[3] = {px - mu4.x, py - mu4.y, pz - mu4.z};
                                float rec32[kRec];
                                for (int x = 0; x < kRec; ++x) rec32[x] = 0.f;
                                // dA += (sum gU0) q^T; dmu = -A^T sum gU0 (+ the view-direction chain)
                                for (int x = 0; x < 3; ++x)
                                    for (int c = 0; c < 3; ++c) rec32[3 * x + c] = fmaf(cb[9 + x], q[c], cb[3 * x + c]);
                                for (int c = 0; c < 3; ++c)
                                    rec32[9 + c] = -(A[c] * cb[9] + A[3 + c] * cb[10] + A[6 + c] * cb[11]);
                                rec32[12] = cb[12];
                                // rho = max(0, 0.5 + f.Y(dir)): the clamp passes where 0.5 + sh >= 0
                                float dx, dy, dz, nrm;
                                view_dir<NLOSGR_PRESET_CUDA>(-q[0], -q[1], -q[2], dx, dy, dz, nrm);
                                float Y[kMaxK];
                                sh_basis<NLOSGR_PRESET_CUDA>(deg, dx, dy, dz, Y);
                                const float* f = fr;
                                const float sh = sh_dot(f, Y, K);
                                const float gr = sh + 0.5f >= 0.f ? cb[13] : 0.f;
                                if (gr != 0.f) {
#pragma unroll
                                    for (int c = 0; c < kMaxK; ++c) rec32[16 + c] = c < K ? gr * Y[c] : 0.f;
                                    float gx, gy, gz;
                                    sh_grad_dir<NLOSGR_PRESET_CUDA>(deg, dx, dy, dz, f, gx, gy, gz);
                                    float ox, oy, oz;
                                    view_dir_bwd<NLOSGR_PRESET_CUDA>(-q[0], -q[1], -q[2], nrm, gr * gx, gr * gy, gr * gz,
                                                                     ox, oy, oz);
                                    rec32[9] += ox; rec32[10] += oy; rec32[11] += oz;
                                }
#pragma unroll
                                for (int x = 0; x < kRec / 4; ++x) {
                                    float4 v = acc4[x];
                                    v.x += rec32[4 * x]; v.y += rec32[4 * x + 1]; v.z += rec32[4 * x + 2]; v.w += rec32[4 * x + 3];
                                    dst[x] = v;
                                }
                            }
                        }
                        if (SEL == NLOSGR_SELECT_AABB) {
                            // cap counters after the window: every staged hit of the ray
                            __syncthreads();
                            if (half == 1)
                                for (int r = rg; r < RT; r += 4) {
                                    const int i = ti0 + r / k.tj, j = tj0 + r % k.tj;
                                    bool h = false;
                                    if (valid && i < nt && j < np_) {
                                        const float dx = sth[i] * cph[j], dy = sth[i] * sph[j], dz = cth[i];
                                        h = slab_hit(sel6, px, py, pz, 1.0f / (dx + 1e-8f), 1.0f / (dy + 1e-8f),
                                                     1.0f / (dz + 1e-8f));
                                    }
                                    const unsigned long long m = __builtin_amdgcn_ballot_w64(h);
                                    if (lane == 0) icnt[r] = min(kCap, icnt[r] + ihalf[r] + __popcll(m));
                                }
                        }
                    }
                    __syncthreads();
                    qh += nst;   // the staged window leaves the queue (the rest moves at the next cull round)
                    TDIAG(trays)
                    if (SEL == NLOSGR_SELECT_AABB) {
                        // the filter keeps the first 256 box hits by index per ray (ray_aabb.cu:10-61) and
                        // windows arrive in index order: once every ray of the tile is full, stop
                        bool full = true;
                        for (int r = 0; r < RT; ++r) {
                            const int i = ti0 + r / k.tj, j = tj0 + r % k.tj;
                            if (i < nt && j < np_ && icnt[r] < kCap) full = false;
                        }
                        if (full) {
                            capped = true;
                            qn = qh = 0;
                            break;
                        }
                    }
                }
            }

            if (!pairs) {
                TDIAG(trays)
                if (!BWD && OCCL && k.rcache) {   // record the (D, W) rows for the backward
                    float2* dst = k.rcache + (size_t)item * RT * nr;
                    for (int x = tid; x < RT * nr; x += kTB) dst[x] = rows[x];
                    __syncthreads();
                }
                // ---------------- scan: wave = ray, lane = bin ----------------
                for (int r = wave; r < RT; r += kTW) {
                    const int i = ti0 + r / k.tj, j = tj0 + r % k.tj;
                    const bool rv = i < nt && j < np_;
                    const float st = rv ? sth[i] : 0.f;
                    const size_t ray = (size_t)p * nt * np_ + (size_t)(rv ? i : 0) * np_ + (rv ? j : 0);
                    float2* row = rows + r * nr;
                    float carry = 0.f;
                    for (int c = 0; c < nch; ++c) {
                        const int kb = c * 64 + lane;
                        const bool in = kb < nr;
                        const float2 dw = in ? row[kb] : make_float2(0.f, 0.f);
                        float out, T = 1.f;
                        if (OCCL) {
                            const float x = dw.x * cdt;
                            const float incl = wave_incl_sum(x);
                            T = fast_exp2(-(carry + incl - x) * kLog2e);
                            out = T >= 1e-4f ? T * dw.y : 0.f;
                            if (!(T >= 1e-4f)) T = 0.f;
                            carry += __shfl(incl, 63);
                        } else {
                            out = dw.y;
                        }
                        if (!BWD) {
                            if (k.ray_out && rv && in) k.ray_out[ray * nr + kb] = out * k.opt.ray_scale;
                            if (in) row[kb].x = rv ? out * st : 0.f;
                        } else {
                            float gk = 0.f;
                            if (rv && in) {
                                if (k.grad_hist) gk = k.grad_hist[(size_t)p * nr + kb] * k.geo.att[kb] * k.geo.hscale[p] * st;
                                if (k.grad_ray) gk += k.grad_ray[ray * nr + kb] * k.opt.ray_scale;
                            }
                            // a = dL/dW; E = dL/dout out (suffix-summed into dL/dD below)
                            if (in) row[kb] = OCCL ? make_float2(gk * T, gk * out) : make_float2(gk, 0.f);
                        }
                    }
                    if (BWD && OCCL) {
                        float suffix = 0.f;
                        for (int c = nch - 1; c >= 0; --c) {
                            const int kb = c * 64 + lane;
                            const bool in = kb < nr;
                            const float E = in ? row[kb].y : 0.f;
                            const float incl = wave_incl_suffix(E);
                            if (in) row[kb].y = -cdt * (suffix + incl - E);
                            suffix += __shfl(incl, 0);
                        }
                    }
                }
                __syncthreads();
                if (!BWD) {
                    float* hp = k.hpart + ((size_t)p * k.ntiles + t) * nr;
                    for (int kb = tid; kb < nr; kb += kTB) {
                        float s = 0.f;
                        for (int r = 0; r < RT; ++r) s += rows[r * nr + kb].x;
                        hp[kb] = s;
                    }
                }
                TDIAG(tscan)
            }
        }
    }
    if (kDiag && k.diag && tid == 0) {
        atomicAdd(k.diag, tcull);
        atomicAdd(k.diag + 1, tstage);
        atomicAdd(k.diag + 2, trays);
        atomicAdd(k.diag + 3, tscan);
        atomicAdd(k.diag + 4, nwin);
        atomicAdd(k.diag + 5, nent);
        atomicAdd(k.diag + 6, nec);
        atomicAdd(k.diag + 7, nchk);
    }
#undef TDIAG
}

// hist[p][k] = (sum over tiles in order) x att[k] x hscale[p]
__global__ __launch_bounds__(256) void tiles_reduce_kernel(const float* __restrict__ hpart, int ntiles, long long P, int nr,
                                                           const float* __restrict__ att, const float* __restrict__ hscale,
                                                           float* __restrict__ hist) {
    const long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= P * nr) return;
    const long long p = x / nr;
    const int kb = (int)(x - p * nr);
    float s = 0.f;
    for (int t = 0; t < ntiles; ++t) s += hpart[(p * ntiles + t) * nr + kb];
    hist[x] = s * att[kb] * hscale[p];
}

// per Gaussian: sum of the slot rows in slot order, chained to the raw parameters
__global__ __launch_bounds__(256) void tiles_finish_kernel(TArgs k, float* d_mu, float* d_scaling, float* d_rot,
                                                           float* d_opac, float* d_feat) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k.g.ng) return;
    float a[kRec];
    for (int x = 0; x < kRec; ++x) a[x] = 0.f;
    for (int s = 0; s < k.nslot; ++s) {
        const float4* src = reinterpret_cast<const float4*>(k.acc + ((size_t)s * k.g.ng + i) * kRec);
        for (int x = 0; x < kRec / 4; ++x) {
            const float4 v = src[x];
            a[4 * x] += v.x; a[4 * x + 1] += v.y; a[4 * x + 2] += v.z; a[4 * x + 3] += v.w;
        }
    }
    d_mu[3 * i] = a[9]; d_mu[3 * i + 1] = a[10]; d_mu[3 * i + 2] = a[11];
    const float sg = 1.0f / (1.0f + expf(-k.g.opacity[i]));
    d_opac[i] = a[12] * sg * (1.0f - sg);
    const int K = (k.g.sh_degree + 1) * (k.g.sh_degree + 1);
    for (int c = 0; c < k.g.k_feat; ++c) d_feat[(size_t)i * k.g.k_feat + c] = c < K ? a[16 + c] : 0.f;
    chain_to_raw<NLOSGR_PRESET_CUDA>(k.g, i, a, d_scaling, d_rot);
}


int cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
    }
    return n;
}

struct TPlan {
    int rt, ti, tj, nti, ntj, ntiles, nslot;
    int pbatch;              // forward: wall points per launch (the tile partials [pbatch][ntiles][nr] stay bounded)
    int bbatch;              // wall points per launch of either sweep (the tile bins [bbatch][ntiles][nwords] too)
    int nwords;              // 64-Gaussian words per tile bin row
    bool bins;               // tile binning on (culled selections; NLOSGR_FLAG_TILE_NOBIN turns it off)
    long long nitems;
    size_t off_cull, off_bbox, off_acc, off_hpart, off_next, off_cones, off_masks, off_rows, total;
};

// tile bins per launch: at most this many bytes (C3: 64 tiles x 1563 words = 800 KB per wall point, so
// 4096-wall-point launches use 3.3 GB; C5's 500k Gaussians x 128 tiles: 524 wall points per launch)
constexpr size_t kBinBytes = (size_t)4 << 30;

// the OCCL row cache: 8 B per (item, tile ray, bin), e.g. C3 (128x128 wall, 32x32 rays, 1024 bins) 128 GiB
bool row_cache(const nlosgr_options* opt) { return opt && opt->ray_cache && opt->mode == NLOSGR_MODE_OCCL; }

TPlan plan(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt) {
    TPlan P;
    P.rt = tile_rays(geo->nr);
    int ti = 1;
    while (ti * ti < P.rt) ti <<= 1;          // TI >= TJ, TI * TJ = RT
    P.ti = ti;
    P.tj = P.rt / ti;
    P.nti = (geo->nt + P.ti - 1) / P.ti;
    P.ntj = (geo->np + P.tj - 1) / P.tj;
    P.ntiles = P.nti * P.ntj;
    P.nitems = (long long)geo->nwall * P.ntiles;
    P.nslot = (int)(P.nitems < cu_count() ? P.nitems : cu_count());
    if (P.nslot < 1) P.nslot = 1;
    const size_t ng = g->ng > 0 ? (size_t)g->ng : 1;
    P.off_cull = align_up(ng * sizeof(GaussRec));
    P.off_bbox = P.off_cull + align_up(ng * sizeof(float4));
    P.off_acc = P.off_bbox + align_up(ng * 6 * sizeof(float));
    P.off_hpart = P.off_acc + align_up((size_t)P.nslot * ng * kRec * sizeof(float));
    // forward tile partials per launch: at most kHpartBytes (C5 with AABB selection: 65536 wall points x
    // 128 tiles x 2048 bins would be 69 GB for the whole wall), so the forward runs in wall-point batches
    const size_t per_wall = (size_t)P.ntiles * geo->nr * sizeof(float);
    const size_t budget = (size_t)(batch_budgets().tile_hpart_mb * 1048576.0);   // default 1 GiB
    long long pb = per_wall ? (long long)(budget / per_wall) : geo->nwall;
    if (pb < 1) pb = 1;
    P.pbatch = (int)(pb < geo->nwall ? pb : geo->nwall);
    if (P.pbatch < 1) P.pbatch = 1;
    P.off_next = P.off_hpart + align_up((size_t)P.pbatch * per_wall);
    // tile binning: every culled selection (AABB boxes, or the support within a cutoff); with a dense support
    // every Gaussian passes every cone, so there is nothing to bin
    P.bins = !(opt->flags & NLOSGR_FLAG_TILE_NOBIN) &&
             (opt->selection == NLOSGR_SELECT_AABB || opt->cutoff > 0.f) && g->ng > 0;
    P.nwords = (int)((ng + 63) / 64);
    const size_t per_wall_bins = P.bins ? (size_t)P.ntiles * P.nwords * sizeof(unsigned long long) : 0;
    long long bb = per_wall_bins ? (long long)(kBinBytes / per_wall_bins) : geo->nwall;
    if (bb < 1) bb = 1;
    P.bbatch = (int)(bb < geo->nwall ? bb : geo->nwall);
    if (P.bbatch < 1) P.bbatch = 1;
    // the launches of both sweeps cover the same wall-point batches (the forward's partials bound it too)
    if (P.pbatch > P.bbatch) P.pbatch = P.bbatch;
    P.off_cones = P.off_next + align_up(sizeof(unsigned long long));
    P.off_masks = P.off_cones + align_up((size_t)P.bbatch * P.ntiles * 8 * sizeof(float));
    P.off_rows = P.off_masks + align_up((size_t)P.bbatch * per_wall_bins);
    P.total = P.off_rows + (row_cache(opt) ? align_up((size_t)P.nitems * P.rt * geo->nr * sizeof(float2)) : 0);
    return P;
}

template <int SEL, bool DENSE, bool OCCL, bool BWD>
void launch_tile(const TArgs& a, size_t shm, hipStream_t s) {
    hipLaunchKernelGGL((tile_kernel<SEL, DENSE, OCCL, BWD>), dim3(a.nslot), dim3(tile_threads<BWD>()), shm, s, a);
}

template <bool BWD>
void dispatch_tile_(const TArgs& a, size_t shm, hipStream_t s);

// NLOSGR_TILES_DIAG=1 (diagnostics only): per-phase cycles of each workgroup's thread 0, printed
template <bool BWD>
void dispatch_tile(const TArgs& a0, size_t shm, hipStream_t s) {
    if (!kDiag || !getenv("NLOSGR_TILES_DIAG")) {
        dispatch_tile_<BWD>(a0, shm, s);
        return;
    }
    TArgs a = a0;
    unsigned long long h[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMalloc(&a.diag, sizeof(h)) != hipSuccess) return;
    (void)hipMemcpyAsync(a.diag, h, sizeof(h), hipMemcpyHostToDevice, s);
    dispatch_tile_<BWD>(a, shm, s);
    (void)hipMemcpyAsync(h, a.diag, sizeof(h), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(a.diag);
    fprintf(stderr, "[tiles %s] slot-cycles cull %.3g stage %.3g windows %.3g scan %.3g windows %llu (slots %d); "
            "wave 0: entries %llu entry-chunks %llu chunks %llu\n",
            BWD ? "bwd" : "fwd", (double)h[0], (double)h[1], (double)h[2], (double)h[3], h[4], a.nslot, h[5], h[6], h[7]);
}

template <bool BWD>
void dispatch_tile_(const TArgs& a, size_t shm, hipStream_t s) {
    const bool occl = a.opt.mode == NLOSGR_MODE_OCCL;
    if (a.opt.selection == NLOSGR_SELECT_AABB) {
        if (occl) launch_tile<NLOSGR_SELECT_AABB, false, true, BWD>(a, shm, s);
        else launch_tile<NLOSGR_SELECT_AABB, false, false, BWD>(a, shm, s);
    } else if (!(a.opt.cutoff > 0.f)) {
        if (occl) launch_tile<NLOSGR_SELECT_SUPPORT, true, true, BWD>(a, shm, s);
        else launch_tile<NLOSGR_SELECT_SUPPORT, true, false, BWD>(a, shm, s);
    } else {
        if (occl) launch_tile<NLOSGR_SELECT_SUPPORT, false, true, BWD>(a, shm, s);
        else launch_tile<NLOSGR_SELECT_SUPPORT, false, false, BWD>(a, shm, s);
    }
}

int prepare(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* ws,
            const TPlan& P, TArgs& a, hipStream_t s) {
    memset(&a, 0, sizeof(a));
    a.g = *g; a.geo = *geo; a.opt = *opt;
    char* base = (char*)ws;
    a.recs = (const GaussRec*)base;
    a.cull = (const float4*)(base + P.off_cull);
    a.bbox = (const float*)(base + P.off_bbox);
    a.acc = (float*)(base + P.off_acc);
    a.hpart = (float*)(base + P.off_hpart);
    a.ti = P.ti; a.tj = P.tj; a.rt = P.rt;
    a.ntile_i = P.nti; a.ntile_j = P.ntj; a.ntiles = P.ntiles;
    a.nitems = P.nitems; a.nslot = P.nslot;
    a.rcache = row_cache(opt) ? (float2*)(base + P.off_rows) : nullptr;
    a.next = (unsigned long long*)(base + P.off_next);
    a.cones = (const float*)(base + P.off_cones);
    a.masks = P.bins ? (const unsigned long long*)(base + P.off_masks) : nullptr;
    a.nwords = P.nwords;
    launch_preprocess(g, (GaussRec*)base, s);
    HIPCHK(hipGetLastError());
    const int nb = (g->ng + 255) / 256;
    if (opt->selection == NLOSGR_SELECT_AABB)
        hipLaunchKernelGGL(cull_prep_kernel<NLOSGR_SELECT_AABB>, dim3(nb), dim3(256), 0, s, *g, a.recs, opt->cutoff,
                           (float4*)a.cull, (float*)a.bbox);
    else
        hipLaunchKernelGGL(cull_prep_kernel<NLOSGR_SELECT_SUPPORT>, dim3(nb), dim3(256), 0, s, *g, a.recs, opt->cutoff,
                           (float4*)a.cull, (float*)a.bbox);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

// the launch arguments of wall points [p0, p0 + pn): geometry tables, the row cache and the items offset
TArgs batch_args(const TArgs& a, const TPlan& P, const nlosgr_geometry* geo, int p0, int pn) {
    const int nt = geo->nt, np_ = geo->np, nr = geo->nr;
    TArgs b = a;
    b.geo.nwall = pn;
    b.geo.wall = geo->wall + 3 * (size_t)p0;
    b.geo.sin_theta = geo->sin_theta + (size_t)p0 * nt;
    b.geo.cos_theta = geo->cos_theta + (size_t)p0 * nt;
    b.geo.sin_phi = geo->sin_phi + (size_t)p0 * np_;
    b.geo.cos_phi = geo->cos_phi + (size_t)p0 * np_;
    b.geo.grid_lin = geo->grid_lin + 4 * (size_t)p0;
    b.geo.hscale = geo->hscale + p0;
    b.nitems = (long long)pn * P.ntiles;
    b.pbase = p0;   // the tile rotation follows the global wall index
    b.nslot = (int)(b.nitems < P.nslot ? b.nitems : P.nslot);
    b.rcache = a.rcache ? a.rcache + (size_t)p0 * P.ntiles * P.rt * nr : nullptr;
    return b;
}

// the batch's tile cones, and its tile bins when binning is on
int bin_batch(const TArgs& b, const TPlan& P, hipStream_t s) {
    const long long nthr = b.nitems * 64;
    hipLaunchKernelGGL(tile_cone_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s, b.geo, P.ti, P.tj,
                       P.ntj, P.ntiles, (float*)b.cones);
    HIPCHK(hipGetLastError());
    if (b.masks) {
        hipLaunchKernelGGL(tile_bin_kernel, dim3((unsigned)((b.g.ng + kBinTB - 1) / kBinTB), (unsigned)b.geo.nwall),
                           dim3(kBinTB), 0, s, b.cull, b.g.ng, b.geo, P.ntiles, P.nwords, b.cones,
                           (unsigned long long*)b.masks);
        HIPCHK(hipGetLastError());
    }
    return NLOSGR_OK;
}

}  // namespace

namespace nlosgr {
namespace detail {

bool tiles_engine(const nlosgr_options* opt) {
    return opt->mode == NLOSGR_MODE_OCCL || opt->selection == NLOSGR_SELECT_AABB;
}

int tiles_validate(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt) {
    if (g->preset != NLOSGR_PRESET_CUDA)
        return set_err(NLOSGR_E_UNSUPPORTED, "occlusion compositing / AABB selection are path C semantics: cuda preset only");
    if (opt->mode != NLOSGR_MODE_OCCL && opt->mode != NLOSGR_MODE_NOOCL)
        return set_err(NLOSGR_E_UNSUPPORTED, "AABB selection supports the noocl and occl modes");
    if (opt->selection != NLOSGR_SELECT_SUPPORT && opt->selection != NLOSGR_SELECT_AABB)
        return set_err(NLOSGR_E_INVALID, "unknown selection");
    if (geo->nr > 4096) return set_err(NLOSGR_E_UNSUPPORTED, "occl / AABB engine: nr <= 4096");
    if ((size_t)TLayout(tile_rays(geo->nr), geo->nr, tile_threads<false>(), false).total * 4 + 16 > 160 * 1024 ||
        (size_t)TLayout(tile_rays(geo->nr), geo->nr, tile_threads<true>(), true).total * 4 + 16 > 160 * 1024)
        return set_err(NLOSGR_E_UNSUPPORTED, "occl / AABB engine: LDS budget");
    return NLOSGR_OK;
}

size_t tiles_workspace_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt) {
    return plan(g, geo, opt).total;
}

int tiles_fwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* ws,
              float* hist_out, float* ray_out, hipStream_t s) {
    if (!ws) return set_err(NLOSGR_E_INVALID, "workspace is null");
    const TPlan P = plan(g, geo, opt);
    if (ray_out) HIPCHK(hipMemsetAsync(ray_out, 0, (size_t)geo->nwall * geo->nt * geo->np * geo->nr * sizeof(float), s));
    if (g->ng == 0) {
        if (hist_out) HIPCHK(hipMemsetAsync(hist_out, 0, (size_t)geo->nwall * geo->nr * sizeof(float), s));
        return NLOSGR_OK;
    }
    TArgs a;
    int rc = prepare(g, geo, opt, ws, P, a, s);
    if (rc) return rc;
    const size_t shm = (size_t)TLayout(P.rt, geo->nr, tile_threads<false>(), false).total * sizeof(float);
    const int nt = geo->nt, np_ = geo->np, nr = geo->nr;
    // wall-point batches: one launch each over the batch's items (pointer offsets into the tables, the
    // outputs and the row cache), so the tile partials and the tile bins stay within their budgets
    for (int p0 = 0; p0 < geo->nwall; p0 += P.pbatch) {
        const int pn = geo->nwall - p0 < P.pbatch ? geo->nwall - p0 : P.pbatch;
        TArgs b = batch_args(a, P, geo, p0, pn);
        b.hist_out = hist_out;
        b.ray_out = ray_out ? ray_out + (size_t)p0 * nt * np_ * nr : nullptr;
        HIPCHK(hipMemsetAsync(b.next, 0, sizeof(unsigned long long), s));
        rc = bin_batch(b, P, s);
        if (rc) return rc;
        dispatch_tile<false>(b, shm, s);
        HIPCHK(hipGetLastError());
        if (hist_out) {
            const long long n = (long long)pn * nr;
            hipLaunchKernelGGL(tiles_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b.hpart,
                               P.ntiles, (long long)pn, nr, geo->att, b.geo.hscale, hist_out + (size_t)p0 * nr);
            HIPCHK(hipGetLastError());
        }
    }
    return NLOSGR_OK;
}

int tiles_bwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* ws,
              const float* grad_hist, const float* grad_ray, float* d_mu, float* d_scaling, float* d_rotation,
              float* d_opacity, float* d_features, hipStream_t s) {
    if (!ws) return set_err(NLOSGR_E_INVALID, "workspace is null");
    const TPlan P = plan(g, geo, opt);
    TArgs a;
    int rc = prepare(g, geo, opt, ws, P, a, s);
    if (rc) return rc;
    a.grad_hist = grad_hist;
    a.grad_ray = grad_ray;
    HIPCHK(hipMemsetAsync(a.acc, 0, (size_t)P.nslot * g->ng * kRec * sizeof(float), s));
    if (geo->nwall > 0 && (grad_hist || grad_ray)) {
        const size_t shm = (size_t)TLayout(P.rt, geo->nr, tile_threads<true>(), true).total * sizeof(float);
        const int nt = geo->nt, np_ = geo->np, nr = geo->nr;
        // the forward's wall-point batches (the row cache's items and the bins' budget); every launch adds into
        // the same slot rows, in batch order
        for (int p0 = 0; p0 < geo->nwall; p0 += P.pbatch) {
            const int pn = geo->nwall - p0 < P.pbatch ? geo->nwall - p0 : P.pbatch;
            TArgs b = batch_args(a, P, geo, p0, pn);
            b.grad_hist = grad_hist ? grad_hist + (size_t)p0 * nr : nullptr;
            b.grad_ray = grad_ray ? grad_ray + (size_t)p0 * nt * np_ * nr : nullptr;
            // with the row cache the workspace holds the forward of these inputs (the rows the backward
            // reloads); when that forward was one launch (one wall-point batch), its tile cones and bins are
            // this batch's too and are not rebuilt
            if (!(a.rcache && P.pbatch >= geo->nwall)) {
                rc = bin_batch(b, P, s);
                if (rc) return rc;
            }
            dispatch_tile<true>(b, shm, s);
            HIPCHK(hipGetLastError());
        }
    }
    hipLaunchKernelGGL(tiles_finish_kernel, dim3((g->ng + 255) / 256), dim3(256), 0, s, a, d_mu, d_scaling, d_rotation,
                       d_opacity, d_features);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

}  // namespace detail
}  // namespace nlosgr

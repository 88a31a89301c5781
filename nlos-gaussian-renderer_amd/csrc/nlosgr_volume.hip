// Transient Gaussian NLOS renderer — volume forward / backward kernels and the C ABI (gfx950).
//
// Hot path: for every relay-wall point p and time bin k
//     hist[p,k] = hscale[p] * att[k] * sum_g w_g(p) sum_{i,j} sin(theta_i) pdf_g(p + r_k d_ij)
// (no-occlusion) or the per-Gaussian self-transmittance variant ('netf').
//
// Algebra that makes the inner loop cheap: with u0 = A(p - mu) and v = A d_ij the whitened
// offset along ray ij is u(r) = u0 + r v, a straight line, so each (pair, ray) is a 1-D
// Gaussian in r:  pdf(r) = exp(-(m2min + a (r - t*)^2) / 2),  a = |v|^2, t* = -(u0.v)/a,
// m2min = |u0 + t* v|^2.  The support |u| <= m_c is
//   * per pair: a cone of rays (bounding-sphere test -> (theta, phi) index box), then
//   * per ray:  the quadric d^T M d >= 0,  M = (A^T u0)(A^T u0)^T - (|u0|^2 - m_c^2) A^T A
//               (exactly m2min <= m_c^2), then
//   * per ray:  one contiguous bin range [kl, kh] (a "segment").
//
// Work decomposition (4 independent waves per workgroup):
//   forward : workgroup = one wall point x a split of the Gaussians.  Lane = (wall point,
//             Gaussian) pair enumerates its candidate rays; passing rays become segments in a
//             wave-private LDS queue.  Lane = segment then walks its bins with the exp2 recurrence
//             and adds them into a wave-private LDS histogram: at the training cutoff as fixed-point
//             integers, two bins per no-return ds_add_u64 (FX drain: no claims, order-independent,
//             exact up to one rounding per term), otherwise as float2 read-add-writes with a claim
//             table keeping the lanes' addresses distinct.  Either way the forward is bitwise
//             deterministic (FX: integer sums; float: fixed-order wave and split reductions).
//   backward: workgroup = 64 Gaussians x a split of the wall; wave w walks wall points
//             w, w+4, ...  Lane = segment runs the bins of one ray serially with its sums in
//             registers; per-pair sums in LDS; per-Gaussian accumulators stay in registers
//             for the whole split and are combined in a fixed order into a partial slab.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#include "nlosgr_common.hpp"

using namespace nlosgr;
using namespace nlosgr::detail;

// A/B switches (compile-time; defaults are the production choice)
// kRecurrence: along a segment the log2 value is quadratic in the bin offset t, e(t) = ga t^2 + al,
// so value(t+1) = value(t) * 2^(ga (2t+1)) and that ratio itself scales by 2^(2 ga) per bin.  The
// culled drains (forward and backward, no-occlusion) re-seed value and ratio with exact exp2 once
// per kSteps-bin round and multiply in between: relative error <= kSteps ulp.  Inside the support
// |ga| t^2 <= m_c^2 log2(e) / 2, which bounds |ga (2t+1)| by m_c^2 log2(e) (<= 47 at m_c = 5.7),
// so the ratio never overflows; past the segment end both factors only shrink (no inf * 0).
// Dense mode (unbounded t) keeps the per-bin exp2.

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct KArgs {
    nlosgr_gaussians g;
    nlosgr_geometry geo;
    nlosgr_options opt;
    const GaussRec* recs;
    float* hist_out;
    float* ray_out;
    const float* grad_hist;
    const float* grad_ray;
    float* partial;  // [nsplit][ng][32]
    int nsplit;
    unsigned long long* counts;  // optional [3]: pairs, segments, samples (nlosgr_count_support)
    ulonglong2* cmask;           // ray cache [P][ng]: passing rays of the pair's box (bit = box cell)
    float* drho;                 // backward: dL/drho per pair [P][ng] (0 outside the support) -> sh_kernel
    float* hpart;                // forward Gaussian-split partial histograms [nfsplit][P][nr]
    float* shpart;               // sh_kernel partials [nsh][ng][kShPart]
    int nsh;                     // sh_kernel wall-point splits
    int nfsplit;                 // forward Gaussian splits per wall point (hpart != null)
    int bshared;                 // backward: 4 waves share each wall point's staged row (bwd_shared)
    unsigned* cbox;              // ray cache [P][ng]: i0 | j0 << 12 | width << 24, 0 = not cached
    float* crho;                 // ray cache [P][ng]: the pair's SH albedo rho (1)
    int g_lo, g_hi;              // backward: Gaussians [g_lo, g_hi) (one bucket of the gradient all-reduce)
    int pb0, pnw;                // backward: wall points [pb0, pb0 + pnw) of this launch (a batch; drho rows
                                 // are indexed p - pb0, so the dL/drho buffer holds one batch, not the wall)
    int accum;                   // backward batches after the first add into the partial slabs
    unsigned long long* hfx;     // forward FX drain: fixed-point histogram [P][nr] (u64, integer adds)
    int* fx_info;                // forward FX drain: [0] unit exponent E (fx_unit_kernel), [1] E of the launch's
                                 // largest bound, [2] LDS flushes, [3] bright segments, [4] bright Gaussians
    const float* fx_bound;       // forward FX drain: amplitude bound per Gaussian [ng] (fx_bound_kernel)
    const int* fx_blist;         // forward FX drain: the bright Gaussians (fx_blist_kernel), [fx_info[4]]
};

// ray cache: a pair whose (theta, phi) candidate box has at most 128 cells records which cells
// passed the quadric test in the forward; the backward walks those bits instead of re-testing
// (C3: 99.9% of pairs; the rest are re-enumerated)
constexpr int kCacheCells = 128;
__device__ __forceinline__ unsigned cache_box(int i0, int j0, int w) {
    return (unsigned)i0 | ((unsigned)j0 << 12) | ((unsigned)w << 24);
}

// atan2 with |error| < 2e-6 rad (minimax on [0,1] + octant reduction); used only for the
// conservative footprint box, which is widened by kAngMargin.
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx > 0.f ? mn * frcp(mx) : 0.f;
    const float s = a * a;
    float r = fmaf(s, -0.01172120f, 0.05265332f);
    r = fmaf(s, r, -0.11643287f);
    r = fmaf(s, r, 0.19354346f);
    r = fmaf(s, r, -0.33262347f);
    r = fmaf(s, r, 0.99997726f);
    r *= a;
    if (ay > ax) r = 1.57079632679f - r;
    if (x < 0.f) r = kPi - r;
    return y < 0.f ? -r : r;
}
constexpr float kAngMargin = 1e-4f;

// 1 - exp(-x) for 0 <= x <= 1/64 as x (1 - x/2 + x^2/6 - x^3/24) (truncation x^4/120 <= 5e-10 relative):
// the netf transmittance factor exp(-sigma pdf c dT) without an exp when c dT <= 1/64 (C3: 1.25e-3;
// sigma <= 1, pdf <= 1), a launch-uniform choice
constexpr float kSmallX = 1.0f / 64.0f;
constexpr float kTf0 = 1.0f + 1e-7f;   // the netf transmittance factor's constant, exp(0) + 1e-7 in float
constexpr float kRTf0 = 1.0f / kTf0;
template <int N>
__device__ __forceinline__ constexpr float kTfPow() {   // kTf0^N (exact in float for small N: 1 + N 2^-23)
    float r = 1.0f;
    for (int i = 0; i < N; ++i) r *= kTf0;
    return r;
}
__device__ __forceinline__ float om_exp_small(float x) {
    return x * fmaf(x, fmaf(x, fmaf(x, -1.0f / 24.0f, 1.0f / 6.0f), -0.5f), 1.0f);
}

// ------------------------------------------------------------------------------------------
// per-(wall point, Gaussian) pair state
// ------------------------------------------------------------------------------------------
struct Pair {
    float A[9], sigma, smax, N[6];
    float q[3];         // p - mu
    float u0[3];        // A (p - mu)
    float dir[3], nrm;  // view direction of mu - p (preset convention)
    float sh, rho, w;
    float M[6];         // quadric (M00, 2M01, 2M02, M11, 2M12, M22)
    int i0, i1, j0, j1;
};

__device__ __forceinline__ void load_rec(const GaussRec& r, Pair& P, float mu[3]) {
    mu[0] = r.a.x; mu[1] = r.a.y; mu[2] = r.a.z; P.sigma = r.a.w;
    P.A[0] = r.b.x; P.A[1] = r.b.y; P.A[2] = r.b.z; P.A[3] = r.b.w;
    P.A[4] = r.c.x; P.A[5] = r.c.y; P.A[6] = r.c.z; P.A[7] = r.c.w;
    P.A[8] = r.d.x; P.smax = r.d.y; P.N[0] = r.d.z; P.N[1] = r.d.w;
    P.N[2] = r.e.x; P.N[3] = r.e.y; P.N[4] = r.e.z; P.N[5] = r.e.w;
}

// f: the Gaussian's feature row (k_feat floats; registers or global)
template <int PRESET, bool DENSE>
__device__ __forceinline__ void pair_setup(const KArgs& k, const float* f, const float mu[3], float px, float py,
                                           float pz, const float* lin, float mc2, Pair& P) {
    P.q[0] = px - mu[0]; P.q[1] = py - mu[1]; P.q[2] = pz - mu[2];
    for (int r = 0; r < 3; ++r) P.u0[r] = P.A[3 * r] * P.q[0] + P.A[3 * r + 1] * P.q[1] + P.A[3 * r + 2] * P.q[2];
    view_dir<PRESET>(-P.q[0], -P.q[1], -P.q[2], P.dir[0], P.dir[1], P.dir[2], P.nrm);
    const float sh = sh_dot<PRESET>(k.g.sh_degree, P.dir[0], P.dir[1], P.dir[2], f);
    P.sh = sh;
    P.rho = fmaxf(sh + 0.5f, 0.0f);
    P.w = P.sigma * P.rho;
    const int nt = k.geo.nt, np_ = k.geo.np;
    P.i0 = 0; P.i1 = nt - 1; P.j0 = 0; P.j1 = np_ - 1;
    if (DENSE) return;
    // quadric cone: d^T M d >= 0  <=>  m2min(d) <= m_c^2
    const float wv0 = P.A[0] * P.u0[0] + P.A[3] * P.u0[1] + P.A[6] * P.u0[2];
    const float wv1 = P.A[1] * P.u0[0] + P.A[4] * P.u0[1] + P.A[7] * P.u0[2];
    const float wv2 = P.A[2] * P.u0[0] + P.A[5] * P.u0[1] + P.A[8] * P.u0[2];
    const float kap = P.u0[0] * P.u0[0] + P.u0[1] * P.u0[1] + P.u0[2] * P.u0[2] - mc2;
    P.M[0] = wv0 * wv0 - kap * P.N[0];
    P.M[1] = 2.0f * (wv0 * wv1 - kap * P.N[1]);
    P.M[2] = 2.0f * (wv0 * wv2 - kap * P.N[2]);
    P.M[3] = wv1 * wv1 - kap * P.N[3];
    P.M[4] = 2.0f * (wv1 * wv2 - kap * P.N[4]);
    P.M[5] = wv2 * wv2 - kap * P.N[5];
    // bounding-sphere cone -> (theta, phi) index box (angles via one fast atan2, widened by a margin)
    const float Rb = k.opt.cutoff * P.smax * 1.0001f + 1e-7f;
    const float dx = -P.q[0], dy = -P.q[1], dz = -P.q[2];
    const float rxy2 = dx * dx + dy * dy;
    const float dist2 = rxy2 + dz * dz;
    const float Rb2 = Rb * Rb;
    if (dist2 <= Rb2) return;
    const float rxy = fsqrt(rxy2);
    const float alpha = fast_atan2(Rb, fsqrt(dist2 - Rb2)) + kAngMargin;       // asin(Rb / dist)
    const float thc = fast_atan2(rxy, dz);                                     // acos(dz / dist)
    const float th0 = lin[0], dth = lin[1], ph0 = lin[2], dph = lin[3];
    if (dth > 0.f) {
        const float idth = frcp(dth);
        // samples are points (theta_i = th0 + i dth): the box holds exactly the samples inside the
        // margin-widened cap range, [ceil(lo), floor(hi)] (floor/ceil added one outside row per side)
        P.i0 = fidx(ceilf((thc - alpha - th0) * idth), 0, nt - 1);
        P.i1 = fidx(floorf((thc + alpha - th0) * idth), -1, nt - 1);
    }
    if (thc - alpha > 1e-3f && thc + alpha < kPi - 1e-3f && dph > 0.f) {
        // max |phi - phi_c| on the cone = asin(sin(alpha) / sin(theta_c))
        const float sa = Rb * frcp(fsqrt(dist2));
        const float sth = rxy * frcp(fsqrt(dist2));
        const float ratio = sa * frcp(sth);
        if (ratio < 0.999f) {
            const float dphi = fast_atan2(ratio, fsqrt(1.0f - ratio * ratio)) + kAngMargin;
            const float phc = fast_atan2(dy, dx);
            const float lo = phc - dphi, hi = phc + dphi;
            if (lo > -kPi && hi < kPi) {
                const float idph = frcp(dph);
                P.j0 = fidx(ceilf((lo - ph0) * idph), 0, np_ - 1);
                P.j1 = fidx(floorf((hi - ph0) * idph), -1, np_ - 1);
            }
        }
    }
}

// feature row -> registers (zero past k_feat)
template <int KM>
__device__ __forceinline__ void load_feat(const nlosgr_gaussians& g, int gi, float* f) {
    const float* src = g.features + (size_t)gi * g.k_feat;
    if (KM % 4 == 0 && g.k_feat == KM && (reinterpret_cast<uintptr_t>(g.features) & 15) == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
        for (int c = 0; c < KM / 4; ++c) {
            const float4 v = s4[c];
            f[4 * c] = v.x; f[4 * c + 1] = v.y; f[4 * c + 2] = v.z; f[4 * c + 3] = v.w;
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < KM; ++c) f[c] = c < g.k_feat ? src[c] : 0.f;
}

__device__ __forceinline__ float quadric(const float* M, float dx, float dy, float dz) {
    const float t0 = fmaf(M[0], dx, fmaf(M[1], dy, M[2] * dz));
    const float t1 = fmaf(M[3], dy, M[4] * dz);
    return fmaf(dx, t0, fmaf(dy, t1, dz * dz * M[5]));
}

// Ray quantities: v = A d, a = |v|^2, t*, z* = u0 + t* v, m2min, in-support bin range, and
// ks = the (fractional) bin of the closest approach.
struct Ray {
    float v[3], a, ts, zs[3], m2min, ks;
    int kl, kh;
};

template <bool DENSE>
__device__ __forceinline__ bool ray_setup(const float* A, const float* u0, float dx, float dy, float dz, float mc2,
                                          float r0, float inv_dr, int nr, Ray& R) {
    for (int r = 0; r < 3; ++r) R.v[r] = A[3 * r] * dx + A[3 * r + 1] * dy + A[3 * r + 2] * dz;
    R.a = R.v[0] * R.v[0] + R.v[1] * R.v[1] + R.v[2] * R.v[2];
    const float b = u0[0] * R.v[0] + u0[1] * R.v[1] + u0[2] * R.v[2];
    const float ia = frcp(R.a);
    R.ts = -b * ia;
    for (int r = 0; r < 3; ++r) R.zs[r] = u0[r] + R.ts * R.v[r];
    R.m2min = R.zs[0] * R.zs[0] + R.zs[1] * R.zs[1] + R.zs[2] * R.zs[2];
    R.ks = (R.ts - r0) * inv_dr;
    if (DENSE) {
        R.kl = 0; R.kh = nr - 1;
        return true;
    }
    if (!(R.m2min <= mc2)) return false;
    const float hk = fsqrt((mc2 - R.m2min) * ia) * inv_dr;
    R.kl = fidx(ceilf(R.ks - hk), 0, nr);
    R.kh = fidx(floorf(R.ks + hk), -1, nr - 1);
    return R.kl <= R.kh;
}

// LDS carve helper (offsets in floats, 16-byte aligned)
__host__ __device__ __forceinline__ int al4(int n) { return (n + 3) & ~3; }

// ray queue ring per wave: < 64 queued + up to 64 (small ring) or 128 appended per enumeration
constexpr int kRQ = 256;
__device__ __forceinline__ unsigned pack_ray(int slot, int i, int j) {
    return (unsigned)slot | ((unsigned)i << 8) | ((unsigned)j << 20);
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// Lane-serial drain: lane = one ray segment, walking its bins kSteps at a time and adding each
// value into the wave-private LDS histogram with a plain read-add-write.  At step m every lane
// touches bin pos + m, so the adds of one instruction hit distinct addresses whenever the lanes'
// start bins differ — guaranteed per round by a claim table (owner[pos] = lane; losers retry
// next round).  Lanes that did not win, or ran past their segment, point at private pad bins
// and add 0, so the step body is branch-free.  Idle lanes are refilled from the ray queue.
#ifndef NLOSGR_FSTEPS
#define NLOSGR_FSTEPS 28
#endif
constexpr int kSteps = NLOSGR_FSTEPS;     // bins per lane per drain round (the largest; netf: kStepsNetf)
#ifndef NLOSGR_FSTEPS_NETF
#define NLOSGR_FSTEPS_NETF 20
#endif
constexpr int kStepsNetf = NLOSGR_FSTEPS_NETF;
static_assert(kStepsNetf <= kSteps && kStepsNetf % 2 == 0, "the layouts' pads hold kSteps bins");
// round 6: 28-bin rounds (with the refill deal at 56 idle lanes and 2 placement claim rounds) for the
// no-occlusion and bin-integrated forwards: C3 734.8 -> 714.4 ms, C4 binint 1150 -> 1090 ms; netf measured
// 883.7 -> 893.8 ms at 28 and keeps 20
template <int MODE>
__device__ __forceinline__ constexpr int fsteps() { return MODE == NLOSGR_MODE_NETF ? kStepsNetf : kSteps; }
#ifndef NLOSGR_REFILL
#define NLOSGR_REFILL 48
#endif
#ifndef NLOSGR_BREFILL
#define NLOSGR_BREFILL 16
#endif
constexpr int kRefill = NLOSGR_REFILL;     // refill once this many lanes are idle (or the queue is final)
#ifndef NLOSGR_REFILL_FX
#define NLOSGR_REFILL_FX 56
#endif
constexpr int kRefillFx = NLOSGR_REFILL_FX;   // the no-occlusion FX drain with the refill deal
constexpr int kBRefill = NLOSGR_BREFILL;   // backward: same rule

#ifndef NLOSGR_FXPERM
#define NLOSGR_FXPERM 1   // FX refill permutation (the deal, see fx_perm): with the bank placement 745.7 vs 750.6 ms
#endif
#ifndef NLOSGR_FXBAL
#define NLOSGR_FXBAL 0    // with NLOSGR_FXPERM: residue balance at refill instead of the placement (fx_balance, opt-in)
#endif
struct FwdLayout {
    int hist, owner, rayq, wave_stride, total;  // offsets in floats
    // fx: the fixed-point drain needs no claim table and no per-lane pad bins (22.7 KB per C3
    // workgroup instead of 26.6 KB: 7 workgroups per CU)
    __host__ __device__ FwdLayout(int nr, int nt, int np_, bool fx = false) {
        const int off = al4(2 * (nt + np_));  // float2 theta table [nt], float2 phi table [np]
        hist = 0;                             // [nr + kSteps] bins + [kSteps + 64] pad bins (fx: [nr + kSteps + 2])
        // fx: the histogram's fields, then 16 residue counters of the refill balance (fx_balance)
        owner = fx ? al4(nr + kSteps + 4) + (NLOSGR_FXPERM && NLOSGR_FXBAL ? 16 : 0) : al4(nr + 2 * kSteps + 64);   // u8 [nr] claim table
        rayq = owner + (fx ? 0 : al4((nr + 3) / 4));   // uint [kRQ] ring
        wave_stride = al4(rayq + kRQ);
        hist += off; owner += off; rayq += off;
        total = off + kWaves * wave_stride;
    }
};

// per-lane drain state (one segment)
struct Drain {
    int pos, rem;     // next bin, bins left
    float t;          // pos - ks (bin offset from the closest approach)
    float ga, al;     // log2 value(t) = ga t^2 + al   (noocl: al includes log2 w [+ log2 sin theta])
    float st;         // sin(theta_i) (kept separate only when per-ray outputs are written)
    float sc, wc, T;      // netf: sigma c dT, w c dT, transmittance T at pos (linear: one exp per bin)
    float beta, xlo, elo; // binint: dr sqrt(a/2), lower bin edge beta (kap - 1/2) and erfc(|xlo|)
    int rbase;        // RAYS: ray * nr
    int wrap;         // dense no-occlusion: bins [0, wrap) still to drain after the first piece [start, nr)
    float tw;         // dense no-occlusion: t at bin 0
};

// Dense no-occlusion segments span every bin, so they would all claim start bin 0 and drain in a
// one-winner-per-round staircase.  Each bin's value is evaluated exactly (no recurrence), so a
// segment may start anywhere: it drains [stag, nr) and then wraps to [0, stag).
template <int MODE, bool DENSE>
__device__ __forceinline__ constexpr bool dense_wrap() { return DENSE && MODE == NLOSGR_MODE_NOOCL; }

template <int MODE, bool DENSE, bool RAYS>
__device__ __forceinline__ bool drain_setup(const float* A, const float* u0, float lw, float sc, float wc,
                                            float2 th, float2 ph, int i, int j, int np_, int nr, float mc2,
                                            float r0, float dr, float inv_dr, float f0log2, Drain& d, int stag = 0) {
    Ray R;
    if (!ray_setup<DENSE>(A, u0, th.x * ph.x, th.x * ph.y, th.y, mc2, r0, inv_dr, nr, R)) return false;
    d.pos = R.kl;
    d.rem = R.kh - R.kl + 1;
    d.t = (float)R.kl - R.ks;
    if (dense_wrap<MODE, DENSE>()) {   // (R.kl, R.kh) = (0, nr - 1)
        d.tw = d.t;
        d.pos = stag;
        d.rem = nr - stag;
        d.wrap = stag;
        d.t = (float)stag - R.ks;
    }

    d.ga = -kHalfLog2e * R.a * dr * dr;
    if (MODE == NLOSGR_MODE_NOOCL) {
        d.al = fmaf(-kHalfLog2e, R.m2min, lw);
        if (!RAYS) d.al += flog2(th.x);
        d.st = th.x;
    } else if (MODE == NLOSGR_MODE_BININT) {
        // bin average of exp(-a (r - t*)^2 / 2) over [r_k -+ dr/2] = sqrt(pi)/(2 beta) (erf(x1) - erf(x0))
        d.beta = dr * sqrtf(0.5f * R.a);
        d.al = fmaf(-kHalfLog2e, R.m2min, lw);   // the erf form's sqrt(pi) / (2 beta) is applied per value
        if (!RAYS) d.al += flog2(th.x);
        d.st = th.x;
        d.xlo = d.beta * (d.t - 0.5f);
        d.elo = erfcf(fabsf(d.xlo));
    } else {
        d.al = -kHalfLog2e * R.m2min;
        d.sc = sc;
        d.wc = RAYS ? wc : wc * th.x;   // histogram-only: sin(theta) folded into the weight
        d.T = fast_exp2((float)R.kl * f0log2);   // (1 + 1e-7)^kl: the empty bins before the segment
        d.st = th.x;
    }
    d.rbase = (i * np_ + j) * nr;
    return true;
}

// Candidate enumeration (lane = pair): quadric test only; passing (pair, ray) entries are appended
// to the ray queue ring at qbase + cnt.  Branch-free body (every lane evaluates a clamped
// candidate, `more` masks the result), two candidates per trip so their table reads overlap;
// returns once cnt >= 64 or every lane exhausted its box (cnt < 64 + 2*64 <= kRQ on return).
template <bool DENSE, bool REC = false>
__device__ __forceinline__ void enumerate_box(const float* M, int i1, int j0, int j1, bool& more, int& ci, int& cj,
                                              const float2* tth, const float2* tph, int nt1, unsigned* rayq,
                                              int qbase, int& cnt, unsigned long long* rec0 = nullptr,
                                              unsigned long long* rec1 = nullptr, int* cell = nullptr) {
    constexpr int NC = 3;
    static_assert(NC >= 1 && 64 + NC * 64 <= kRQ, "enumeration would overflow the ray queue ring");
    const int lane = lane_id();
    do {
        // NC consecutive cells of the box (row-major): all table reads are issued before any queue
        // store (an LDS store in between would order them), the tests are unpredicated
        int cis[NC], cjs[NC];
        bool mores[NC];
        cis[0] = ci; cjs[0] = cj; mores[0] = more;
#pragma unroll
        for (int u = 1; u < NC; ++u) {
            const bool wrap = cjs[u - 1] >= j1;
            cis[u] = cis[u - 1] + (wrap ? 1 : 0);
            cjs[u] = wrap ? j0 : cjs[u - 1] + 1;
            mores[u] = mores[u - 1] & (cis[u] <= i1);
        }
        float2 ths[NC], phs[NC];
#pragma unroll
        for (int u = 0; u < NC; ++u) { ths[u] = tth[min(cis[u], nt1)]; phs[u] = tph[cjs[u]]; }
        bool pass[NC];
#pragma unroll
        for (int u = 0; u < NC; ++u)
            pass[u] = mores[u] & (DENSE || quadric(M, ths[u].x * phs[u].x, ths[u].x * phs[u].y, ths[u].y) >= 0.f);
        if (REC) {   // cell index within the box (only boxes of <= 128 cells are cached)
            const int c0 = *cell;
#pragma unroll
            for (int u = 0; u < NC; ++u) {
                const int cu = c0 + u;
                *rec0 |= (pass[u] & (cu < 64)) ? (1ull << (cu & 63)) : 0ull;
                *rec1 |= (pass[u] & ((cu >> 6) == 1)) ? (1ull << (cu & 63)) : 0ull;
            }
            *cell = c0 + NC;
        }
        unsigned es[NC];
#pragma unroll
        for (int u = 0; u < NC; ++u) es[u] = pack_ray(lane, cis[u], cjs[u]);
        {
            const bool wrap = cjs[NC - 1] >= j1;
            cj = wrap ? j0 : cjs[NC - 1] + 1;
            ci = cis[NC - 1] + (wrap ? 1 : 0);
            more = mores[NC - 1] & (ci <= i1);
        }
        int at = cnt;
#pragma unroll
        for (int u = 0; u < NC; ++u) {
            const unsigned long long m = __builtin_amdgcn_ballot_w64(pass[u]);
            if (pass[u]) rayq[(qbase + at + lanes_below(m)) & (kRQ - 1)] = es[u];
            at += __popcll(m);
        }
        cnt = at;
    } while (cnt < 64 && __builtin_amdgcn_ballot_w64(more));
}

// Ray-cache walk (backward): each lane pops the lowest set cell of its pair's cached mask and
// appends that ray; same queue discipline as enumerate_box (no quadric, no table reads).
__device__ __forceinline__ void enumerate_cached(unsigned long long& bits0, unsigned long long& bits1, int ci0,
                                                 int cj0, int cw, float rcw, unsigned* rayq, int qbase, int& cnt) {
    const int lane = lane_id();
    do {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const bool lo = bits0 != 0ull;
            const bool pass = lo || bits1 != 0ull;
            const int b = lo ? (int)__builtin_ctzll(bits0) : (pass ? 64 + (int)__builtin_ctzll(bits1) : 0);
            if (lo) bits0 &= bits0 - 1ull;
            else bits1 &= bits1 - 1ull;
            const int di = (int)(((float)b + 0.5f) * rcw);
            const unsigned e = pack_ray(lane, ci0 + di, cj0 + b - di * cw);
            const unsigned long long m = __builtin_amdgcn_ballot_w64(pass);
            if (pass) rayq[(qbase + cnt + lanes_below(m)) & (kRQ - 1)] = e;
            cnt += __popcll(m);
        }
    } while (cnt < 64 && __builtin_amdgcn_ballot_w64((bits0 | bits1) != 0ull));
}

__device__ __forceinline__ void compiler_fence() { __asm__ __volatile__("" ::: "memory"); }

// TAIL (culled histogram at cutoff >= kTailCutoff): the forward drain has no end mask.  A round adds
// kSteps values from the even bin at or below pos (a bin before pos, o = 1, adds 0): the bins past the
// segment's end (up to kSteps - 1) get their exact Gaussian values, each < exp(-m_c^2 / 2) of the
// Gaussian's peak (<= 3.7e-6 at m_c >= kTailCutoff), so the result lies between the culled and the
// dense sum.  Bins past nr land in the zeroed pad row.
constexpr float kTailCutoff = 5.0f;
// debug build (-DNLOSGR_FCOUNT, scripts/drain_counts.py): count_support runs the TAIL forward and returns
// (wave drain rounds, active lanes summed over rounds, claim winners summed) instead of its work counts
#ifdef NLOSGR_FCOUNT
#define NLOSGR_FCOUNT_ON 1
#else
#define NLOSGR_FCOUNT_ON 0
#endif
constexpr float kBetaSeries = 0.5f;   // bin-integrated TAIL drain: series bin average up to this beta

// Fixed-point drain (FX; TAIL no-occlusion histogram, the training hot path).  The wave's LDS histogram
// holds each bin as an unsigned 32-bit count of units 2^-E; a round adds two bins per lane with ONE
// no-return ds_add_u64 of the packed pair (low word = even bin, high word = odd bin), so no claim table:
// every active lane drains every round, and integer adds make the sum independent of the order (the
// forward is bitwise deterministic whatever the schedule).  A value rounds to the nearest unit
// (v_cvt_rpi_i32_f32).
// The unit (round 6): E is set per launch from the amplitude bounds b_g = sigma_g * rho_max_g of the
// Gaussians (fx_bound_kernel; rho_max by Cauchy-Schwarz on the SH bands) so that the bound of the
// ceil(ng/256)-th brightest Gaussian is < 2^kFxBits units (fx_unit_kernel, a quantile over the bounds'
// binary exponents), not the largest bound: a few very bright Gaussians no longer coarsen the unit of
// all the others (round 5 used the maximum, so 0.1 % of Gaussians 10^3-10^4 x brighter than the rest cost
// the rest 10-13 bits, and their sub-half-unit tails rounded to zero: a one-sided bias).  A segment whose
// peak is >= 2^kFxBits units at refill ("bright"; at most the segments of the ceil(ng/256) Gaussians above
// the quantile, and none unless the bounds spread by more than the C-S slack) bypasses the LDS: its lane
// adds its values as u64 integers straight into the wall point's global u64 row (agent-scope atomics), so
// it is as exact as the rest.  E is clamped to <= E(max bound) + range, range = kFxRange or less when
// (bright Gaussians <= ceil(ng / 256)) x (rays per wall point) bright terms per bin could pass 2^(63 - kFxBits -
// range): the u64 sums cannot wrap (C3 / C5: range 16, at most 2^19 / 2^21 bright terms of < 2^40 units).
// A low word must never carry into its high word: every lane sums the peaks (exp2 of the segment's log2
// amplitude, in units) of the LDS segments it took since the last check; a segment adds at most its peak
// to any bin once, so while every lane's sum stays <= thr the largest field stays <= M + 64 thr < 2^32.
// When a lane passes thr the wave reads its histogram's true maximum M; past 2^31 it moves the fields into
// the u64 row in global memory (integer atomics) and zeroes them.  At the end each workgroup adds its 4
// waves' fields to the global u64 histogram [P][nr] (all Gaussian splits of a wall point meet there), and
// fx_reduce_kernel scales it to floats.
#ifdef NLOSGR_FXCOUNT
__device__ unsigned long long g_fdbg[8];
#endif
constexpr int kFxBits = 24;
constexpr int kFxRange = 16;                 // E <= E(max bound) + kFxRange: u64 terms < 2^(kFxBits + kFxRange)
constexpr float kFxBright = 16777216.0f;     // 2^kFxBits
constexpr float kFxMargin = 1.002f;          // segment peak <= bound x 2^E x kFxMargin (binint 1.001, netf (1+1e-7)^nr)
constexpr float kFxLimit = 4294967040.0f;   // largest float below 2^32
constexpr int kFxBins = 256;                 // bound histogram: one bin per binary exponent (float bits >> 23)
constexpr int kFxTailBytes = 2048;           // workspace tail of the FX area: bins u32 [256] | info int [8]
// FX bank placement.  A ds_add_u64 is serviced in 4 groups of 16 lanes; two lanes of a group whose words lie
// on the same bank pair (word index mod 16) serialize.  Every active lane advances 10 words per round, so the
// pairs' residues within a group stay fixed for a segment's life: at refill a new segment may start up to
// kFxShift words (2 bins each) early, on the nearest residue no older lane of its group holds and no lower
// new lane of the group takes (3 claim rounds of row-wide DPP ORs; a segment that finds none keeps its
// start).  The early bins get the Gaussian's exact values (as the TAIL overrun past the end), only while the
// recurrence's seed stays >= 2^-100 units.  Placement never affects correctness, only conflicts.
#ifndef NLOSGR_FXSHIFT
#define NLOSGR_FXSHIFT 4
#endif
constexpr int kFxShift = NLOSGR_FXSHIFT;
#ifndef NLOSGR_FXPLACE_ROUNDS
#define NLOSGR_FXPLACE_ROUNDS 2
#endif
constexpr int kFxPlaceRounds = NLOSGR_FXPLACE_ROUNDS;   // claim rounds of the refill placement
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ unsigned row_or(unsigned x) {   // OR over the lane's 16-lane row
    x |= dpp_u<0x121>(x);   // row_ror:1
    x |= dpp_u<0x122>(x);   // row_ror:2
    x |= dpp_u<0x124>(x);   // row_ror:4
    x |= dpp_u<0x128>(x);   // row_ror:8
    return x;
}
__device__ __forceinline__ unsigned row_or_below(unsigned x) {   // OR over the lanes below in the row
    x |= dpp_u<0x111>(x);   // row_shr:1 (lanes shifted in read 0)
    x |= dpp_u<0x112>(x);
    x |= dpp_u<0x114>(x);
    x |= dpp_u<0x118>(x);
    return dpp_u<0x111>(x);
}

// round to nearest (floor(x + 0.5)) as an integer in one VALU instruction; 0 <= x < 2^31
__device__ __forceinline__ unsigned cvt_rpi(float x) {
    int r;
    __asm__("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return (unsigned)r;
}
// two bins of a TAIL drain round into the wave's LDS histogram: FX = one packed fixed-point ds_add_u64
// (values in units), otherwise a float2 read-add-write (the claim table keeps the lanes' pairs distinct)
template <bool FX>
__device__ __forceinline__ void emit2(float2* at, float v0, float v1) {
    if (FX) {
        const unsigned long long pv = ((unsigned long long)cvt_rpi(v1) << 32) | cvt_rpi(v0);
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(at), pv, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
    } else {
        float2 x = *at;
        x.x += v0; x.y += v1;
        *at = x;
        __asm__ __volatile__("" ::: "memory");
    }
}

// FX bright segment: one value (in units, rounded to nearest; non-finite saturates) as a u64 integer add
// into the wall point's global row (agent-scope atomic, no return)
__device__ __forceinline__ void fx_gadd(unsigned long long* at, float v) {
    const unsigned long long u = (unsigned long long)fminf(v + 0.5f, 1.8e19f);
    __hip_atomic_fetch_add(at, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// FX refill placement (see kFxShift): newl = this lane took a new segment, act = it holds one
__device__ __forceinline__ void fx_place(bool newl, bool act, Drain& d) {
    if (!__builtin_amdgcn_ballot_w64(newl)) return;
    const int pb = d.pos >> 1, ph = pb & 15, o = d.pos & 1;
    unsigned occ = row_or((act && !newl) ? (1u << ph) : 0u);
    // reach: the seed exponent at the new start stays >= -100 (no flush to zero), the start >= bin 0
    const float span = d.al + 100.f;
    const float tm = span > 0.f ? __builtin_amdgcn_sqrtf(span * __builtin_amdgcn_rcpf(fmaxf(-d.ga, 1e-30f))) : 0.f;
    const int smax = newl ? min(min(kFxShift, pb), (int)floorf(0.5f * (d.t - (float)o + tm))) : -1;
    bool pend = newl && smax >= 0;
    int sh = 0;
#pragma unroll
    for (int it = 0; it < kFxPlaceRounds; ++it) {
        const unsigned fm = ~occ & 0xFFFFu;
        const unsigned x = ((fm << (15 - ph)) | (fm >> (ph + 1))) & 0xFFFFu;   // bit 15 - k = residue ph - k
        const int dd = x ? (int)__builtin_clz(x) - 16 : 16;
        const bool want = pend && dd <= smax;
        const unsigned bit = want ? 1u << ((ph - dd) & 15) : 0u;
        const bool won = want && !(row_or_below(bit) & bit);
        if (won) sh = dd;
        pend = pend && want && !won;
        occ |= row_or(won ? bit : 0u);
        if (!__builtin_amdgcn_ballot_w64(pend)) break;
    }
    if (sh > 0) {
        const int delta = o + 2 * sh;
        d.pos -= delta;
        d.rem += delta;
        d.t -= (float)delta;
    }
}

// FX refill balance (no-occlusion FX drain, with the deal below).  The deal leaves a group cost of about
// ceil(c / 4) for a residue held by c segments, so the largest residue count sets the ds_add_u64 conflicts
// (scripts/fx_counts.py).  At refill each new segment may start up to kFxShift words early (exact Gaussian
// values before its support, as fx_place): it takes the smallest shift whose residue holds fewer than
// ceil(active / 16) segments, claimed with a wave-private LDS counter per residue (ds_add_rtn; a claim past
// the cap is undone and the next shift tried; none free: no shift).  Placement affects only conflicts.
__device__ __forceinline__ void fx_balance(bool newl, bool act, Drain& d, unsigned* cnt) {
    const int lane = lane_id();
    if (lane < 16) cnt[lane] = 0u;
    wave_sync();
    const int pb = d.pos >> 1, o = d.pos & 1;
    if (act && !newl)
        __hip_atomic_fetch_add(cnt + (pb & 15), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    wave_sync();
    const unsigned cap = (unsigned)((__popcll(__builtin_amdgcn_ballot_w64(act)) + 15) >> 4);
    // reach: the seed exponent at the new start stays >= -100 (no flush to zero), the start >= bin 0
    const float span = d.al + 100.f;
    const float tm = span > 0.f ? __builtin_amdgcn_sqrtf(span * __builtin_amdgcn_rcpf(fmaxf(-d.ga, 1e-30f))) : 0.f;
    const int smax = newl ? min(min(kFxShift, pb), (int)floorf(0.5f * (d.t - (float)o + tm))) : -1;
    int sh = -1;
#pragma unroll
    for (int s2 = 0; s2 <= kFxShift; ++s2) {
        const bool tryit = newl && sh < 0 && s2 <= smax;
        if (!__builtin_amdgcn_ballot_w64(tryit)) break;
        if (tryit) {
            unsigned* c = cnt + ((pb - s2) & 15);
            const unsigned v = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            if (v < cap) sh = s2;
            else __hip_atomic_fetch_add(c, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
    }
    wave_sync();
    if (sh > 0) {
        const int delta = o + 2 * sh;
        d.pos -= delta;
        d.rem += delta;
        d.t -= (float)delta;
    }
}

// FX refill permutation (no-occlusion FX drain).  Every active lane advances the same kSteps / 2 words per
// round, so the bank pair (word mod 16) of each segment relative to the others is fixed for its life: the
// conflicts of a ds_add_u64 (serviced in 4 groups of 16 lanes, bank pair = word mod 16; scripts/lds_fx_probe.hip
// modes 11-16) are set by which segments share a 16-lane group.  At refill the segments are re-dealt over the
// lanes: sorted by (residue, lane) with the idle lanes last, and position s goes to lane 16 (s mod 4) + s / 4,
// so the segments of one residue land in different groups (a residue held by c segments costs ceil(c / 4) per
// group, the least any assignment can reach) and the active lanes spread evenly over the groups.  The sort is
// bit-serial over ballots (5 key bits, no per-residue tables); the state moves with ds_permute (a bijection).
// The per-lane headroom sums (fxs) stay: their total still bounds every field.
#ifndef NLOSGR_FX_DIAG_NOCONFLICT
#define NLOSGR_FX_DIAG_NOCONFLICT 0
#endif
constexpr bool kFxPerm = NLOSGR_FXPERM != 0;   // (defaults with FwdLayout above)
#ifndef NLOSGR_FXPERM_NETF
#define NLOSGR_FXPERM_NETF 0   // measured: netf fwd 894.5 vs 884.5 ms without (its drain is less LDS-bound)
#endif
constexpr bool kFxPermNetf = NLOSGR_FXPERM_NETF != 0;
template <int MODE>
__device__ __forceinline__ void fx_perm(bool& newl, bool& act, Drain& d, float& fpk) {
    const unsigned res = (unsigned)((d.pos >> 1) & 15);
    // deal: sorted by (residue, lane), idle lanes last; position s -> lane 16 (s mod 4) + s / 4
    const unsigned key = act ? res : 16u;
    unsigned long long eq = ~0ull, lt = 0ull;
#pragma unroll
    for (int b = 4; b >= 0; --b) {
        const bool mine = (key >> b) & 1u;
        const unsigned long long B = __builtin_amdgcn_ballot_w64(mine);
        lt |= mine ? (eq & ~B) : 0ull;
        eq &= mine ? B : ~B;
    }
    const int s = __popcll(lt) + lanes_below(eq);
    const int dst = ((s & 3) << 4) | (s >> 2);
    const int a4 = dst << 2;
    const int ri = act ? (d.rem | (newl ? (1 << 30) : 0)) : 0;
    const int ri2 = __builtin_amdgcn_ds_permute(a4, ri);
    d.pos = __builtin_amdgcn_ds_permute(a4, d.pos);
    d.t = __int_as_float(__builtin_amdgcn_ds_permute(a4, __float_as_int(d.t)));
    d.ga = __int_as_float(__builtin_amdgcn_ds_permute(a4, __float_as_int(d.ga)));
    d.al = __int_as_float(__builtin_amdgcn_ds_permute(a4, __float_as_int(d.al)));
    fpk = __int_as_float(__builtin_amdgcn_ds_permute(a4, __float_as_int(fpk)));
    if (MODE == NLOSGR_MODE_NETF) {   // the segment's transmittance (carrying its weight) and sigma c dT
        d.T = __int_as_float(__builtin_amdgcn_ds_permute(a4, __float_as_int(d.T)));
        d.sc = __int_as_float(__builtin_amdgcn_ds_permute(a4, __float_as_int(d.sc)));
    }
    act = ri2 != 0;
    newl = (ri2 >> 30) & 1;
    d.rem = ri2 & ((1 << 30) - 1);
}

// One TAIL drain round of a lane's segment (the QUADF histograms at cutoff >= kTailCutoff): kSteps values from
// the even bin at or below pos (slot 0 before pos adds 0 in a segment's first round), every pair of bins to
// emit(kv, v0, v1); t = d.t, T = the round's copy of d.T (netf: updated).  The drain rounds emit into the LDS
// histogram, or (the bright launch, BR) the wall point's global u64 row.
constexpr int kVW = 2;   // bins per LDS access of the vector drain (float2 / packed u64)
template <int MODE, class Emit>
__device__ __forceinline__ void tail_round(const Drain& d, const float t, float& T, Emit&& emit) {
    const int o = d.pos & (kVW - 1);
    if (MODE == NLOSGR_MODE_NOOCL) {
        // the recurrence is seeded at pos (inside the support: a seed one bin further out can
        // underflow for Gaussians much narrower than a bin); slot 0 before pos (o = 1) adds 0
        float cur = fast_exp2(fmaf(d.ga, t * t, d.al));
        float q = fast_exp2(d.ga * fmaf(2.f, t, 1.f));
        const float cc = fast_exp2(2.f * d.ga);
        {
#pragma unroll
            for (int kv = 0; kv < fsteps<MODE>() / kVW; ++kv) {
                const float v0 = (kv == 0 && o) ? 0.f : cur;
                if (kv == 0) {
                    cur = o ? cur : cur * q;
                    q = o ? q : q * cc;
                } else {
                    cur *= q;
                    q *= cc;
                }
                const float v1 = cur;
                cur *= q;
                q *= cc;
                emit(kv, v0, v1);
            }
        }
    } else if (MODE == NLOSGR_MODE_BININT) {
        // bin-integrated (C4), TAIL: the average of exp(-beta^2 t^2) over the bin [t - 1/2, t + 1/2]
        // (t in bins from the closest approach, beta = dr sqrt(a / 2)) is g(t) (1 + sum_n g^(2n)(t) /
        // (2^2n (2n+1)!) / g(t)) = g(t) P(beta^2 t^2), P a cubic from the n <= 3 terms: relative error
        // <= 7e-8 for beta <= kBetaSeries (a Gaussian wider than 1.4 bins along the ray), so g comes
        // from the exp2 recurrence as in the numerical drain and each bin costs a cubic instead of
        // two erfc.  Narrower rays (beta > kBetaSeries) take the erf difference, when a round holds one.
        const float b = d.beta * d.beta;
        const float c3 = b * b * b * (1.0f / 5040.0f);
        const float c2 = b * b * fmaf(b, -1.0f / 672.0f, 1.0f / 120.0f);
        const float c1 = b * fmaf(b, fmaf(b, 1.0f / 448.0f, -1.0f / 40.0f), 1.0f / 6.0f);
        const float c0 = fmaf(b, fmaf(b, fmaf(b, -1.0f / 2688.0f, 1.0f / 160.0f), -1.0f / 12.0f), 1.0f);
        const float t0 = t - (float)o;    // t of slot 0
        float cur = fast_exp2(fmaf(d.ga, t * t, d.al));
        float q = fast_exp2(d.ga * fmaf(2.f, t, 1.f));
        const float cc = fast_exp2(2.f * d.ga);
        const bool series = d.beta <= kBetaSeries;
        const bool anyerf = __builtin_amdgcn_ballot_w64(!series) != 0;   // (EXEC = the winners)
        const float pref = fast_exp2(d.al) * (0.88622692545275801f * frcp(d.beta));
        {
#pragma unroll
            for (int kv = 0; kv < fsteps<MODE>() / kVW; ++kv) {
                float v[kVW];
#pragma unroll
                for (int jj = 0; jj < kVW; ++jj) {
                    const int jslot = kVW * kv + jj;
                    const float tj = t0 + (float)jslot;
                    const float u = b * tj * tj;
                    float val = cur * fmaf(u, fmaf(u, fmaf(u, c3, c2), c1), c0);
                    if (anyerf && !series) {
                        const float x0 = d.beta * (tj - 0.5f), x1 = d.beta * (tj + 0.5f);
                        const float e0 = erfcf(fabsf(x0)), e1 = erfcf(fabsf(x1));
                        const float df = x0 >= 0.f ? e0 - e1 : (x1 <= 0.f ? e1 - e0 : 2.0f - e0 - e1);
                        val = pref * df;
                    }
                    const bool pre = kv == 0 && jj < o;   // slot before pos (first round of a segment)
                    v[jj] = pre ? 0.f : val;
                    cur = pre ? cur : cur * q;
                    q = pre ? q : q * cc;
                }
                emit(kv, v[0], v[1]);
            }
        }
    } else {
        // netf, TAIL: out_k = w c dT sin(theta) pdf_k T_k, T_{k+1} = T_k (exp(-sigma pdf_k c dT)
        // + 1e-7), two bins per float2 read-add-write; slot 0 before pos (o = 1, a segment's
        // first round) adds 0 and leaves T as it is
        float cur = fast_exp2(fmaf(d.ga, t * t, d.al));   // seeded at pos (see above)
        // the recurrence runs on p~_m = pdf_m c0^m and the transmittance on T~_m = T_m / c0^m (m = bins
        // past pos, c0 = kTf0 = 1 + 1e-7): v_m = T~_m p~_m = T_m pdf_m and T~_{m+1} = T~_m f_m / c0 =
        // T~_m + v_m g(p~_m) with g the cubic's p-terms over c0, one fma per bin (T rescaled per round)
        float q = fast_exp2(d.ga * fmaf(2.f, t, 1.f)) * kTf0;
        const float cc = fast_exp2(2.f * d.ga);
        // the TAIL netf forward runs only at c dT <= kSmallX, so x = sigma pdf c dT <= 1/64 and
        // exp(-x) + 1e-7 is the cubic the backward uses (truncation x^4 / 24 <= 2.5e-9): no exp.
        // As a cubic in pdf: f = c0 + e1 pdf + e2 pdf^2 + e3 pdf^3, e1 = -sx, e2 = sx^2 / 2, e3 =
        // -sx^3 / 6 (the 1e-7 folded into c0: 1 + 1e-7 rounds to 1 + 2^-23, 1.9e-8 per bin); g takes
        // p~ for pdf, 1 + 2.4e-6 relative at most within a round: f off by <= 2.4e-6 x per bin
        const float sx = d.sc;
        const float e1 = -sx * kRTf0, e2 = 0.5f * sx * sx * kRTf0, e3 = (-1.0f / 6.0f) * sx * sx * sx * kRTf0;
        auto gfac = [e1, e2, e3](float pv) { return fmaf(pv, fmaf(pv, e3, e2), e1); };
        {
#pragma unroll
            for (int kv = 0; kv < fsteps<MODE>() / kVW; ++kv) {
                const float p0 = cur;
                if (kv == 0) {
                    cur = o ? cur : cur * q;
                    q = o ? q : q * cc;
                } else {
                    cur *= q;
                    q *= cc;
                }
                const float p1 = cur;
                cur *= q;
                q *= cc;
                // T carries w c dT sin(theta) (set at the segment's start); slot 0 before pos adds 0
                // and (v0 = 0) leaves T as it is
                const float v0 = (kv == 0 && o) ? 0.f : T * p0;
                T = fmaf(v0, gfac(p0), T);
                const float v1 = T * p1;
                T = fmaf(v1, gfac(p1), T);
                emit(kv, v0, v1);
            }
        }
        T *= o ? kTfPow<fsteps<MODE>() - 1>() : kTfPow<fsteps<MODE>()>();   // T = T~ c0^(bins advanced)
    }
}

template <int PRESET, int MODE, bool DENSE, bool RAYS, bool CACHE, bool TAIL, bool FX, bool BR = false>
__device__ __forceinline__ void fwd_body(const KArgs& k) {
    extern __shared__ __align__(16) float smem[];
    const int nr = k.geo.nr, nt = k.geo.nt, np_ = k.geo.np;
    const FwdLayout L(nr, nt, np_, FX);
    static_assert(!FX || (TAIL && !DENSE && !RAYS), "fixed-point drain: TAIL histogram drains only");
    float2* tth = reinterpret_cast<float2*>(smem);
    float2* tph = tth + nt;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();   // wave-uniform (SGPR)
    float* wb = smem + wave * L.wave_stride;
    float* hist = wb + L.hist;
    unsigned char* owner = reinterpret_cast<unsigned char*>(wb + L.owner);
    unsigned* rayq = reinterpret_cast<unsigned*>(wb + L.rayq);
    const int p = blockIdx.x;
    // Gaussian split of this wall point (grid.y; 64-aligned ranges): partial histograms are summed
    // in split order by hist_reduce_kernel when gridDim.y > 1
    const int gsplit = blockIdx.y, nsp = gridDim.y;
    // BR (the bright launch): the Gaussians of the bright list instead of all of them
    const int gcount = BR ? k.fx_info[4] : k.g.ng;
    const int gper = (((gcount + nsp - 1) / nsp) + 63) & ~63;
    const int g_lo = gsplit * gper, g_hi = min(gcount, g_lo + gper);

    for (int t = threadIdx.x; t < nt; t += blockDim.x)
        tth[t] = make_float2(k.geo.sin_theta[(size_t)p * nt + t], k.geo.cos_theta[(size_t)p * nt + t]);
    for (int t = threadIdx.x; t < np_; t += blockDim.x)
        tph[t] = make_float2(k.geo.cos_phi[(size_t)p * np_ + t], k.geo.sin_phi[(size_t)p * np_ + t]);
    for (int t = lane; t < (FX ? nr + kSteps + 4 : nr + 2 * kSteps + 64); t += 64) hist[t] = 0.f;
    __syncthreads();

    const float px = k.geo.wall[3 * p], py = k.geo.wall[3 * p + 1], pz = k.geo.wall[3 * p + 2];
    const float* lin = k.geo.grid_lin + 4 * (size_t)p;
    const float mc2 = k.opt.cutoff * k.opt.cutoff;
    const float r0 = k.geo.r[0];
    const float dr = nr > 1 ? (k.geo.r[nr - 1] - r0) / (float)(nr - 1) : 0.f;
    const float inv_dr = dr > 0.f ? 1.0f / dr : 0.f;
    const float cdt = k.opt.c_deltaT;
    const float f0log2 = log2f(1.0f + 1e-7f);
    float* rout = RAYS ? k.ray_out + (size_t)p * nt * np_ * nr : nullptr;
    const float rscale = k.opt.ray_scale;
    const int flags = k.opt.flags;
    // FX: log2 of the unit scale, folded into every pair's log2 amplitude; per-lane peak bookkeeping
    const float fxE = FX ? (float)k.fx_info[0] : 0.f;
    const float fxS = FX ? fast_exp2(fxE) : 1.f;   // exact: fxE is an integer
    float fthr = kFxLimit / 64.f;   // wave-uniform
    float fpk = 0.f, fxs = 0.f;     // this lane's segment peak, and its peaks since the last check
    unsigned long long* const grow = FX ? k.hfx + (size_t)p * nr : nullptr;
    unsigned* hist32 = reinterpret_cast<unsigned*>(hist);
    const int nfx = nr + kSteps + 2;   // fields a round can reach (bins past nr are pad)
    // the float2 drain (two bins per LDS read-add-write; claim keys on bin pairs)
    constexpr bool QUADF = (MODE == NLOSGR_MODE_NOOCL || ((MODE == NLOSGR_MODE_NETF || MODE == NLOSGR_MODE_BININT) && TAIL)) &&
                           !RAYS && !DENSE;
    const int pad = nr + kSteps + lane;       // this lane's private pad bins (non-winners)
    const int padq = al4(nr + kSteps);        // quad drain: one pad quad row shared by non-winners (they add 0)
    unsigned npair = 0, nseg = 0;
    unsigned long long nsamp = 0;

#ifdef NLOSGR_FXCOUNT
    unsigned long long fdbg[5] = {0ull, 0ull, 0ull, 0ull, 0ull};   // wave-uniform diagnostics
#endif
    Drain d;
    d.pos = 0; d.rem = 0; d.t = 0.f; d.ga = 0.f; d.al = 0.f; d.st = 0.f;
    d.sc = 0.f; d.wc = 0.f; d.T = 0.f; d.rbase = 0;
    d.beta = 0.f; d.xlo = 0.f; d.elo = 0.f;
    d.wrap = 0; d.tw = 0.f;
    bool act = false;
    int qhead = 0, qcount = 0;

    constexpr int VW = kVW;

    for (int base = g_lo + wave * 64;; base += kBlock) {
        const bool have = base < g_hi;         // wave-uniform
        Pair P;
        float lw = 0.f, sc = 0.f, wc = 0.f;
        bool more = false;
        int ci = 0, cj = 0;
        unsigned long long crec0 = 0ull, crec1 = 0ull;   // CACHE: passing cells of this lane's box
        int ccell = 0;
        P.i0 = P.i1 = P.j0 = P.j1 = 0;
        if (have) {
            const int gi = base + lane;
            // the record is loaded ahead of the setup math; the SH coefficients are read from global
            // inside the albedo sum (a register copy of the row spilled the setup at 80 VGPRs)
            const int gl = BR ? k.fx_blist[min(gi, g_hi - 1)] : min(gi, k.g.ng - 1);
            const GaussRec nrec = k.recs[gl];
            // FX: Gaussians whose bound reaches 2^kFxBits units (bright, see kFxBits) are the bright launch's:
            // preprocess_kernel stored them with a negative sigma (the same comparison as fx_blist_kernel), so
            // here w <= 0 skips them; the bright launch takes |sigma|
            if (gi < g_hi) {
                float mu[3];
                load_rec(nrec, P, mu);
                if (BR) P.sigma = fabsf(P.sigma);
                pair_setup<PRESET, DENSE>(k, k.g.features + (size_t)gl * k.g.k_feat, mu, px, py, pz, lin, mc2, P);
                more = (P.w > 0.f) && P.i0 <= P.i1 && P.j0 <= P.j1;
                lw = more ? flog2(P.w) + fxE : 0.f;
                sc = P.sigma * cdt;
                wc = more ? P.w * cdt * fxS : 0.f;   // netf: the value's scale rides on T
            }
            if (flags & 2) more = false;      // diagnostics: pair setup only
            npair += NLOSGR_FCOUNT_ON ? 0u : (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(more));
            ci = P.i0; cj = P.j0;
        }
        while (true) {
            if (qcount < 64 && __builtin_amdgcn_ballot_w64(more)) {
                wave_sync();
                enumerate_box<DENSE, CACHE>(P.M, P.i1, P.j0, P.j1, more, ci, cj, tth, tph, nt - 1, rayq, qhead,
                                            qcount, &crec0, &crec1, &ccell);
                wave_sync();
            }
            const bool anymore = __builtin_amdgcn_ballot_w64(more) != 0;
            const unsigned long long idle = __builtin_amdgcn_ballot_w64(!act);
            const int nidle = __popcll(idle);
            // the no-occlusion FX drain refills later: the deal's cost is per refill (REFILL 48 / 52 / 56 / 60 / 62:
            // 745.9 / 735.7 / 732.4 / 736.7 / 745.4 ms, same box)
            constexpr int kRef = (FX && !BR && ((kFxPerm && MODE == NLOSGR_MODE_NOOCL) ||
                                                (kFxPermNetf && MODE == NLOSGR_MODE_NETF))) ? kRefillFx : kRefill;
            if (qcount > 0 && (nidle >= kRef || !anymore)) {
                // idle lane of rank r takes queue entry qhead + r; pair data come from lane `slot`
                const int r = lanes_below(idle);
                const bool take = !act && r < qcount;
                const unsigned e = take ? rayq[(qhead + r) & (kRQ - 1)] : 0u;
                const int slot = e & 0xFF, i = (e >> 8) & 0xFFF, j = e >> 20;
                float A[9], u0[3];
#pragma unroll
                for (int c = 0; c < 9; ++c) A[c] = __shfl(P.A[c], slot);
#pragma unroll
                for (int c = 0; c < 3; ++c) u0[c] = __shfl(P.u0[c], slot);
                const float lws = __shfl(lw, slot);
                const float scs = MODE == NLOSGR_MODE_NETF ? __shfl(sc, slot) : 0.f;
                const float wcs = MODE == NLOSGR_MODE_NETF ? __shfl(wc, slot) : 0.f;
                bool got = false;
                if (take && !(flags & 1)) {
                    // dense: consecutive queue entries start 37 bins apart (distinct claim keys)
                    const int stag = dense_wrap<MODE, DENSE>() ? (int)(((unsigned)(qhead + r) * 37u) % (unsigned)nr) : 0;
                    got = drain_setup<MODE, DENSE, RAYS>(A, u0, lws, scs, wcs, tth[i], tph[j], i, j, np_, nr, mc2,
                                                         r0, dr, inv_dr, f0log2, d, stag);
                    if (got && !NLOSGR_FCOUNT_ON) nsamp += (unsigned)(d.rem + (dense_wrap<MODE, DENSE>() ? d.wrap : 0));
                    if (MODE == NLOSGR_MODE_NETF && TAIL && QUADF) d.T *= d.wc;   // the weight rides on T
                    act = got && !(flags & 4);    // diagnostics: segment records only
                    if (FX && act) {
                        // the segment's largest value (t = 0), in units (netf: T <= its start x (1 + 1e-7)^nr)
                        fpk = MODE == NLOSGR_MODE_NETF ? d.T * fast_exp2(d.al) * 1.001f
                                                       : fast_exp2(d.al) * (MODE == NLOSGR_MODE_BININT ? 1.001f : 1.f);
                        fxs += fpk;
                    }
                }
                nseg += NLOSGR_FCOUNT_ON ? 0u : (unsigned)__popcll(__builtin_amdgcn_ballot_w64(got));
                const int ntake = min(nidle, qcount);
                qhead = (qhead + ntake) & (kRQ - 1);
                qcount -= ntake;
                // (netf keeps its start: its transmittance would have to be re-seeded)
                bool newl = take && act;
                if (FX && !BR && NLOSGR_FXBAL && kFxPerm && kFxShift > 0 && MODE == NLOSGR_MODE_NOOCL)
                    fx_balance(newl, act, d, reinterpret_cast<unsigned*>(hist + al4(nr + kSteps + 4)));
                // netf has no refill placement (its transmittance would need re-seeding); the deal is opt-in
                // there too (NLOSGR_FXPERM_NETF)
                if (FX && !BR && ((kFxPerm && MODE == NLOSGR_MODE_NOOCL) || (kFxPermNetf && MODE == NLOSGR_MODE_NETF)))
                    fx_perm<MODE>(newl, act, d, fpk);
                if (FX && !BR && kFxShift > 0 && MODE != NLOSGR_MODE_NETF && !(NLOSGR_FXBAL && kFxPerm && MODE == NLOSGR_MODE_NOOCL))
                    fx_place(newl, act, d);
            }
            const bool anyact = __builtin_amdgcn_ballot_w64(act) != 0;
            if (!anyact) {
                if (!anymore && qcount == 0) break;
                continue;
            }
            if (!anymore && qcount == 0 && have) break;   // next Gaussians; segments carry over
            // claim distinct start keys (distinct addresses; vector drain: distinct start pairs)
            constexpr bool QUAD = QUADF;
            bool win = act;   // FX: integer adds, no claims
            if (FX && !BR && __builtin_amdgcn_ballot_w64(fxs > fthr)) {
                // a lane passed its share of the headroom: read the fields' true maximum (and move
                // them to the global u64 histogram once it passes 2^31)
                wave_sync();
                unsigned mx = 0u;
                for (int t = lane; t < nfx; t += 64) mx = max(mx, hist32[t]);
                for (int o2 = 32; o2 > 0; o2 >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o2));
                if (mx >= 0x80000000u) {
                    if (lane == 0) atomicAdd(k.fx_info + 2, 1);
                    for (int t = lane; t < nfx; t += 64) {
                        const unsigned v = hist32[t];
                        if (v && t < nr)
                            __hip_atomic_fetch_add(k.hfx + (size_t)p * nr + t, (unsigned long long)v, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                        hist32[t] = 0u;
                    }
                    wave_sync();
                    mx = 0u;
                }
                fthr = (kFxLimit - (float)mx) * (1.0f / 64.0f);
                fxs = act ? fpk : 0.f;   // an active segment may still add up to its peak to any bin
            }
            if (!FX) {
                const int key = QUAD ? (d.pos / VW) : d.pos;
                if (act) owner[key] = (unsigned char)lane;
                wave_sync();
                win = act && owner[key] == (unsigned char)lane;
                wave_sync();
            }
            if (NLOSGR_FCOUNT_ON) {
                npair += 1u;
                nseg += (unsigned)__popcll(__builtin_amdgcn_ballot_w64(act));
                nsamp += (unsigned)__popcll(__builtin_amdgcn_ballot_w64(win));   // every lane: / 64 on the host
            }
#ifdef NLOSGR_FXCOUNT
            if (FX && !BR) {   // diagnostics: bank-pair occupancy of this round's ds_add_u64 groups
                const unsigned res = (unsigned)((d.pos >> 1) & 15);
                unsigned long long same = __builtin_amdgcn_ballot_w64(act);
                for (int b = 0; b < 4; ++b) {
                    const unsigned long long B = __builtin_amdgcn_ballot_w64((res >> b) & 1u);
                    same &= ((res >> b) & 1u) ? B : ~B;
                }
                const unsigned long long gm = 0xFFFFull << (lane & 48);
                int cg = act ? __popcll(same & gm) : 0;     // lanes of my group on my bank pair
                for (int o2 = 1; o2 < 16; o2 <<= 1) cg = max(cg, __shfl_xor(cg, o2));
                int cw = act ? __popcll(same) : 0;
                for (int o2 = 1; o2 < 64; o2 <<= 1) cw = max(cw, __shfl_xor(cw, o2));
                unsigned rm = act ? (1u << res) : 0u;
                for (int o2 = 1; o2 < 64; o2 <<= 1) rm |= (unsigned)__shfl_xor((int)rm, o2);
                int sg = 0;
                for (int g4 = 0; g4 < 4; ++g4) sg += __shfl(cg, 16 * g4);
                const int na = __popcll(__builtin_amdgcn_ballot_w64(act));
                fdbg[0] += 1ull; fdbg[1] += (unsigned long long)na; fdbg[2] += (unsigned long long)sg;
                fdbg[3] += (unsigned long long)__popc(rm); fdbg[4] += (unsigned long long)cw;
            }
#endif
            const int remw = win ? d.rem : 0;
            float* hb = hist + (win ? (QUAD ? (d.pos & ~(VW - 1)) : d.pos) : (QUAD ? padq : pad));
            float t = d.t;
            float T = d.T;
            float xlo = d.xlo, elo = d.elo;
            if (QUAD) {
                // kSteps bins from the even bin at or below pos: one ds_read_b64 + ds_write_b64 per 2
                // bins, values by the exp2 recurrence (see kRecurrence).  Slots before pos (first round
                // of a segment only) add 0 and do not advance the recurrence, which starts at pos.
                // The whole round is one EXEC region of the winners (losers take no LDS bank and no
                // per-step mask switching).
                const int o = d.pos & (VW - 1);
                const int lim = remw + o;   // slot j is in the segment iff o <= j < lim
                if (TAIL && win) {
                    // (FX: every emitting lane is a winner, so its row starts at the even bin with no loser select)
#if NLOSGR_FX_DIAG_NOCONFLICT   // diagnostics (wrong sums): every lane on its own word residue, no bank conflicts
                    float2* const hbw = reinterpret_cast<float2*>(FX ? hist + 2 * lane : hb);
#else
                    float2* const hbw = reinterpret_cast<float2*>(FX ? hist + (d.pos & ~(VW - 1)) : hb);
#endif
                    if (BR) {   // bright launch: u64 integer adds straight into the wall point's global row
                        const int gb0 = d.pos & ~(VW - 1);
                        tail_round<MODE>(d, t, T, [&](int kv, float v0, float v1) {
                            const int b = gb0 + VW * kv;
                            if (b < nr && v0 > 0.f) fx_gadd(grow + b, v0);
                            if (b + 1 < nr && v1 > 0.f) fx_gadd(grow + b + 1, v1);
                        });
                    } else {
                        tail_round<MODE>(d, t, T, [&](int kv, float v0, float v1) { emit2<FX>(hbw + kv, v0, v1); });
                    }
                } else if (win) {
                    float cur = fast_exp2(fmaf(d.ga, t * t, d.al));
                    float q = fast_exp2(d.ga * fmaf(2.f, t, 1.f));
                    const float cc = fast_exp2(2.f * d.ga);
                    float2* hb2 = reinterpret_cast<float2*>(hb);
#pragma unroll
                    for (int kv = 0; kv < fsteps<MODE>() / VW; ++kv) {
                        float v[VW];
#pragma unroll
                        for (int jj = 0; jj < VW; ++jj) {
                            const int j = VW * kv + jj;
                            if (kv == 0) {
                                const bool st = jj >= o;
                                v[jj] = (st && j < lim) ? cur : 0.f;
                                cur = st ? cur * q : cur;
                                q = st ? q * cc : q;
                            } else {
                                v[jj] = j < lim ? cur : 0.f;
                                cur *= q;
                                q *= cc;
                            }
                        }
                        float2 x = hb2[kv];
                        x.x += v[0]; x.y += v[1];
                        hb2[kv] = x;
                        compiler_fence();
                    }
                }
                t += (float)(fsteps<MODE>() - o);
            } else {
            // netf, culled: pdf by the exp2 recurrence (kRecurrence), re-seeded per round
            constexpr bool REC = MODE == NLOSGR_MODE_NETF && !DENSE;
            const float nsc = -d.sc * (2.f * kHalfLog2e);   // exp(-sigma c dT pdf) = exp2(pdf nsc)
            float cur = 0.f, rq = 0.f, rcc = 0.f;
            if (REC) {
                cur = fast_exp2(fmaf(d.ga, t * t, d.al));
                rq = fast_exp2(d.ga * fmaf(2.f, t, 1.f));
                rcc = fast_exp2(2.f * d.ga);
            }
#pragma unroll
            for (int m = 0; m < fsteps<MODE>(); ++m) {
                const bool in = m < remw;
                const float e2 = fmaf(d.ga, t * t, d.al);
                float v;
                if (MODE == NLOSGR_MODE_NOOCL) {
                    const float pv = fast_exp2(e2);
                    v = in ? pv : 0.f;
                    if (RAYS) {
                        if (in) atomicAdd(rout + d.rbase + d.pos + m, rscale * pv);
                        v *= d.st;
                    }
                } else if (MODE == NLOSGR_MODE_BININT) {
                    // erf(x1) - erf(x0) from erfc of |x| (no cancellation in the tails)
                    const float x1 = d.beta * (t + 0.5f);
                    const float e1 = erfcf(fabsf(x1));
                    const float df = xlo >= 0.f ? elo - e1 : (x1 <= 0.f ? e1 - elo : 2.0f - elo - e1);
                    xlo = x1;
                    elo = e1;
                    const float pv = fast_exp2(d.al) * (0.88622692545275801f * frcp(d.beta)) * df;
                    v = in ? pv : 0.f;
                    if (RAYS) {
                        if (in) atomicAdd(rout + d.rbase + d.pos + m, rscale * pv);
                        v *= d.st;
                    }
                } else {
                    // T_k = prod_{k' < k} (exp(-sigma pdf_k' c dT) + 1e-7), out_k = w c dT pdf_k T_k
                    float pdf;
                    if (REC) {
                        pdf = cur;
                        cur *= rq;
                        rq *= rcc;
                    } else {
                        pdf = fast_exp2(e2);
                    }
                    const float f = fast_exp2(pdf * nsc) + 1e-7f;
                    const float val = d.wc * T * pdf;
                    if (RAYS && in) atomicAdd(rout + d.rbase + d.pos + m, rscale * val);
                    T *= in ? f : 1.f;
                    v = in ? (RAYS ? val * d.st : val) : 0.f;
                }
                t += 1.f;
                const float x = hb[m];
                hb[m] = x + v;
                compiler_fence();
            }
            }
            if (win) {
                const int adv = QUAD ? fsteps<MODE>() - (d.pos & (VW - 1)) : fsteps<MODE>();
                d.t = t;
                d.T = T;
                d.xlo = xlo;
                d.elo = elo;
                d.pos += adv;
                d.rem -= adv;
                if (dense_wrap<MODE, DENSE>() && d.rem <= 0 && d.wrap > 0) {   // second piece [0, wrap)
                    d.pos = 0;
                    d.rem = d.wrap;
                    d.wrap = 0;
                    d.t = d.tw;
                }
                act = d.rem > 0;
            }
        }
        if (CACHE && have && base + lane < g_hi) {
            // every candidate of this chunk has been tested: record the pair's passing cells
            const int bw = P.j1 - P.j0 + 1, bh = P.i1 - P.i0 + 1;
            const bool live = P.w > 0.f && bw > 0 && bh > 0;
            const size_t o = (size_t)p * k.g.ng + base + lane;
            const bool ok = !live || bw * bh <= kCacheCells;
            k.cmask[o] = live ? make_ulonglong2(crec0, crec1) : make_ulonglong2(0ull, 0ull);
            k.cbox[o] = ok ? cache_box(live ? P.i0 : 0, live ? P.j0 : 0, live ? bw : 1) : 0u;
            k.crho[o] = live ? P.rho : 0.f;
        }
        if (!have) break;
    }
    if (k.counts) {
        unsigned long long ns = nsamp;
        for (int o = 32; o > 0; o >>= 1) ns += __shfl_xor(ns, o);
        if (lane == 0) {
            atomicAdd(k.counts, (unsigned long long)npair);
            atomicAdd(k.counts + 1, (unsigned long long)nseg);
            atomicAdd(k.counts + 2, ns);
        }
    }
#ifdef NLOSGR_FXCOUNT
    if (lane == 0)
        for (int c = 0; c < 5; ++c) atomicAdd(&g_fdbg[c], fdbg[c]);
#endif
    if (BR) {   // bright segments taken (nlosgr_fx_info)
        if (lane == 0 && nseg) atomicAdd(k.fx_info + 3, (int)nseg);
        return;
    }
    __syncthreads();
    if (FX) {
        // the 4 waves' fields of each bin -> one integer add into the wall point's global u64 row
        for (int t = threadIdx.x; t < nr; t += blockDim.x) {
            unsigned long long s = 0ull;
            for (int w = 0; w < kWaves; ++w)
                s += reinterpret_cast<const unsigned*>(smem + w * L.wave_stride + L.hist)[t];
            if (s) __hip_atomic_fetch_add(k.hfx + (size_t)p * nr + t, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (k.hist_out) {
        const float hs = k.geo.hscale[p];
        for (int t = threadIdx.x; t < nr; t += blockDim.x) {
            float s = 0.f;
            for (int w = 0; w < kWaves; ++w) s += smem[w * L.wave_stride + L.hist + t];
            if (nsp > 1)
                k.hpart[((size_t)gsplit * k.geo.nwall + p) * nr + t] = s;
            else
                k.hist_out[(size_t)p * nr + t] = s * k.geo.att[t] * hs;
        }
    }
}

template <int PRESET, int MODE, bool DENSE, bool RAYS, bool CACHE, bool TAIL = false, bool FX = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 8))) void fwd_kernel(KArgs k) {
    fwd_body<PRESET, MODE, DENSE, RAYS, CACHE, TAIL, FX>(k);
}
// FX bright launch (BR): the Gaussians whose amplitude bound reaches 2^kFxBits units (fx_blist_kernel), every
// segment added as u64 integers straight into the wall point's global row (kFxBits); usually an empty list
template <int PRESET, int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 8))) void fx_bright_kernel(KArgs k) {
    fwd_body<PRESET, MODE, false, false, false, true, true, true>(k);
}
// nlosgr_count_support's launch of the same body under its own name, so profiles tell it apart from the
// timed forward by identity
template <int PRESET, int MODE, bool DENSE, bool TAIL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6, 8))) void count_kernel(KArgs k) {
    fwd_body<PRESET, MODE, DENSE, false, false, TAIL, false>(k);
}

// forward Gaussian splits: hist[p,t] = (sum over splits in order) x att[t] x hscale[p]
__global__ __launch_bounds__(kBlock) void hist_reduce_kernel(const float* __restrict__ hpart, int nsp, long long P,
                                                             int nr, const float* __restrict__ att,
                                                             const float* __restrict__ hscale, float* __restrict__ hist) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P * nr) return;
    const long long p = i / nr;
    const int t = (int)(i - p * nr);
    float s = 0.f;
    for (int sp = 0; sp < nsp; ++sp) s += hpart[(size_t)sp * P * nr + i];
    hist[i] = s * att[t] * hscale[p];
}

// FX: each Gaussian's amplitude bound b_g = sigma_g * rho_max_g, rho_max = 0.5 + sum_l |f_l| sqrt((2l+1)/4pi)
// (Cauchy-Schwarz with sum_m Y_lm(d)^2 = (2l+1)/4pi on the unit sphere; 5 % margin for the cuda preset's
// eps-shortened view direction), counted into a histogram of binary exponents (float bits >> 23; a
// workgroup histogram in LDS first, then its non-empty bins into the global one).  Non-finite or zero
// bounds are not counted: a NaN Gaussian is skipped by the drains (w > 0 fails) and must not move the unit
// of the others; an infinite one takes the bright path (saturating, kFxBits).
template <int PRESET>
__global__ __launch_bounds__(kBlock) void fx_bound_kernel(nlosgr_gaussians g, float ascale, unsigned* bins,
                                                         float* bound) {
    __shared__ unsigned lh[kFxBins];
    lh[threadIdx.x] = 0u;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < g.ng) {
        const float sig = 1.0f / (1.0f + expf(-g.opacity[i]));
        const float* f = g.features + (size_t)i * g.k_feat;
        const int deg = min(g.sh_degree, PRESET == NLOSGR_PRESET_TORCH ? 4 : 3);
        float sh = 0.f;
        for (int l = 0; l <= deg; ++l) {
            float n2 = 0.f;
            for (int c = l * l; c < (l + 1) * (l + 1) && c < g.k_feat; ++c) n2 += f[c] * f[c];
            sh += sqrtf(n2) * sqrtf((2.0f * l + 1.0f) * (0.25f / kPi));
        }
        const float a = sig * (0.5f + 1.05f * sh) * 1.001f * ascale;   // ascale: the mode's factor (netf: c dT)
        if (a > 0.f && a < 3.0e38f) atomicAdd(&lh[__float_as_uint(a) >> 23], 1u);
        // per Gaussian: 0 for NaN (skipped everywhere), +inf past the float range (the bright launch saturates)
        bound[i] = a >= 3.0e38f ? INFINITY : (a > 0.f ? a : 0.f);
    }
    __syncthreads();
    const unsigned c = lh[threadIdx.x];
    if (c) atomicAdd(bins + threadIdx.x, c);
}

// FX: the unit exponent from the bound histogram (one workgroup).  e_q = the largest exponent bin with at
// least ceil(n / 256) counted bounds at or above it (bin e holds bounds in [2^(e-127), 2^(e-126))), so
// fewer than ceil(n / 256) Gaussians have a bound above 2^(e_q - 126); E = kFxBits - (e_q - 126) puts that
// bound below 2^kFxBits units.  E <= E(top bin) + kFxRange.  info[0] = E, info[1] = E of the top bin.
__global__ __launch_bounds__(kFxBins) void fx_unit_kernel(const unsigned* __restrict__ bins, int* info, int maxunit,
                                                         int range) {
    __shared__ unsigned cum[kFxBins];
    const int t = threadIdx.x;
    cum[t] = bins[t];
    __syncthreads();
    for (int off = 1; off < kFxBins; off <<= 1) {   // suffix sums: cum[e] = sum_{e' >= e} bins[e']
        const unsigned v = t + off < kFxBins ? cum[t + off] : 0u;
        __syncthreads();
        cum[t] += v;
        __syncthreads();
    }
    const unsigned n = cum[0];
    const unsigned kq = (n + 255u) / 256u;
    // the largest e with cum[e] >= kq (resp. >= 1 for the top bin): cum is non-increasing in e
    const bool q = n > 0u && cum[t] >= kq && (t + 1 == kFxBins || cum[t + 1] < kq);
    const bool top = n > 0u && cum[t] >= 1u && (t + 1 == kFxBins || cum[t + 1] < 1u);
    __shared__ int eq, et;
    if (t == 0) { eq = 0; et = 0; }
    __syncthreads();
    if (q) eq = t;
    if (top) et = t;
    __syncthreads();
    if (t == 0) {
        auto unit = [](int e) { const int u = kFxBits - (e - 126); return u < -120 ? -120 : (u > 120 ? 120 : u); };
        const int emax = n > 0u ? unit(et) : 0;
        int e = n > 0u ? unit(maxunit ? et : eq) : 0;   // maxunit: round 5's rule (diagnostics)
        if (e > emax + range) e = emax + range;
        info[0] = e;
        info[1] = emax;
    }
}

// FX: the bright Gaussians (bound x 2^E x kFxMargin >= 2^kFxBits, the comparison of fwd_body) appended to a
// list (any order: the bright launch's sums are integers); info[4] = their number
__global__ __launch_bounds__(kBlock) void fx_blist_kernel(const float* __restrict__ bound, int ng, int* info, int* blist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ng) return;
    const float fxS = ldexpf(1.0f, info[0]);
    if (!(bound[i] * fxS * kFxMargin < kFxBright)) blist[atomicAdd(info + 4, 1)] = i;
}

// FX: hist[p,t] = (u64 count x 2^-E) x att[t] x hscale[p]
__global__ __launch_bounds__(kBlock) void fx_reduce_kernel(const unsigned long long* __restrict__ hfx,
                                                           const int* __restrict__ info, long long P, int nr,
                                                           const float* __restrict__ att,
                                                           const float* __restrict__ hscale, float* __restrict__ hist) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P * nr) return;
    const long long p = i / nr;
    const int t = (int)(i - p * nr);
    const double q = ldexp(1.0, -info[0]);
    hist[i] = (float)((double)hfx[i] * q) * att[t] * hscale[p];
}

// Dense no-occlusion forward (cutoff <= 0: every Gaussian at every sample, the reference's own
// support): every ray covers every bin, so the lane-serial drain above degenerates (all segments
// claim the same bins; read-add-write chains bound by LDS latency).  Here lane = bin instead: a
// wave walks its live pairs one at a time, computes 64 rays of the pair lane-parallel (lane = ray),
// stages their (gamma, alpha, ks) in LDS and then, ray by ray (LDS broadcast), every lane adds the
// exact value of its NB bins (k = lane + 64 b) into register accumulators.  No LDS writes in the
// inner loop, no claims, fixed summation order (deterministic).
struct FwdDenseLayout {
    int rays, hist, total;   // offsets in floats after the float2 angle tables
    __host__ __device__ FwdDenseLayout(int nr, int nt, int np_) {
        const int off = al4(2 * (nt + np_));
        rays = off;                     // float4 [kWaves][64] (gamma, alpha, ks, -)
        hist = rays + kWaves * 64 * 4;  // double [kWaves][nr]
        total = hist + kWaves * nr * 2;
    }
};

template <int PRESET, int NB>
__global__ __launch_bounds__(kBlock) void fwd_dense_kernel(KArgs k) {
    extern __shared__ __align__(16) float smem[];
    const int nr = k.geo.nr, nt = k.geo.nt, np_ = k.geo.np;
    const FwdDenseLayout L(nr, nt, np_);
    float2* tth = reinterpret_cast<float2*>(smem);
    float2* tph = tth + nt;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();   // wave-uniform (SGPR)
    float4* rp = reinterpret_cast<float4*>(smem + L.rays) + wave * 64;
    const int p = blockIdx.x;
    const int gsplit = blockIdx.y, nsp = gridDim.y;
    const int gper = (((k.g.ng + nsp - 1) / nsp) + 63) & ~63;
    const int g_lo = gsplit * gper, g_hi = min(k.g.ng, g_lo + gper);
    for (int t = threadIdx.x; t < nt; t += blockDim.x)
        tth[t] = make_float2(k.geo.sin_theta[(size_t)p * nt + t], k.geo.cos_theta[(size_t)p * nt + t]);
    for (int t = threadIdx.x; t < np_; t += blockDim.x)
        tph[t] = make_float2(k.geo.cos_phi[(size_t)p * np_ + t], k.geo.sin_phi[(size_t)p * np_ + t]);
    __syncthreads();

    const float px = k.geo.wall[3 * p], py = k.geo.wall[3 * p + 1], pz = k.geo.wall[3 * p + 2];
    const float* lin = k.geo.grid_lin + 4 * (size_t)p;
    const float r0 = k.geo.r[0];
    const float dr = nr > 1 ? (k.geo.r[nr - 1] - r0) / (float)(nr - 1) : 0.f;
    const float inv_dr = dr > 0.f ? 1.0f / dr : 0.f;
    const int nray = nt * np_;
    // each 64-ray batch's terms are summed in fp32 registers (<= 64 terms per bin) and folded into the
    // lane's own bins of a wave-private fp64 histogram: a running fp32 total over every (Gaussian, ray)
    // drops the terms below half an ulp of the bin (C2: 1.9e-5 low against float64)
    double* wh = reinterpret_cast<double*>(smem + L.hist) + wave * nr;
    float kf[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        kf[b] = (float)(lane + 64 * b);
        if (lane + 64 * b < nr) wh[lane + 64 * b] = 0.0;
    }

    for (int base = g_lo + wave * 64; base < g_hi; base += kBlock) {
        const int gi = base + lane;
        Pair P;
        float lw = 0.f;
        bool live = false;
        {
            const int gl = min(gi, k.g.ng - 1);
            const GaussRec rec = k.recs[gl];
            float mu[3];
            load_rec(rec, P, mu);
            pair_setup<PRESET, true>(k, k.g.features + (size_t)gl * k.g.k_feat, mu, px, py, pz, lin, 0.f, P);
            live = gi < g_hi && P.w > 0.f;
            lw = live ? flog2(P.w) : 0.f;
        }
        unsigned long long lm = __builtin_amdgcn_ballot_w64(live);
        while (lm) {   // wave-uniform walk over the chunk's live pairs
            const int sl = (int)__builtin_ctzll(lm);
            lm &= lm - 1ull;
            float A[9], u0[3];
#pragma unroll
            for (int c = 0; c < 9; ++c) A[c] = __shfl(P.A[c], sl);
#pragma unroll
            for (int c = 0; c < 3; ++c) u0[c] = __shfl(P.u0[c], sl);
            const float lws = __shfl(lw, sl);
            for (int rb = 0; rb < nray; rb += 64) {
                const int ray = min(rb + lane, nray - 1);
                const int i = ray / np_, j = ray - i * np_;
                const float2 th = tth[i], ph = tph[j];
                Ray R;
                ray_setup<true>(A, u0, th.x * ph.x, th.x * ph.y, th.y, 0.f, r0, inv_dr, nr, R);
                const float ga = -kHalfLog2e * R.a * dr * dr;
                const float al = fmaf(-kHalfLog2e, R.m2min, lws) + flog2(th.x);
                wave_sync();   // the previous batch's broadcasts are done
                rp[lane] = make_float4(ga, al, R.ks, 0.f);
                wave_sync();
                const int nq = min(64, nray - rb);
                float acc[NB];
#pragma unroll
                for (int b = 0; b < NB; ++b) acc[b] = 0.f;
                int q = 0;
                for (; q + 4 <= nq; q += 4) {
                    float4 e[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) e[u] = rp[q + u];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int b = 0; b < NB; ++b) {
                            const float t = kf[b] - e[u].z;
                            acc[b] += fast_exp2(fmaf(e[u].x, t * t, e[u].y));
                        }
                }
                for (; q < nq; ++q) {
                    const float4 e = rp[q];
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        const float t = kf[b] - e.z;
                        acc[b] += fast_exp2(fmaf(e.x, t * t, e.y));
                    }
                }
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    if (lane + 64 * b < nr) wh[lane + 64 * b] += (double)acc[b];
            }
        }
    }
    __syncthreads();
    const float hs = k.geo.hscale[p];
    const double* whs = reinterpret_cast<const double*>(smem + L.hist);
    for (int t = threadIdx.x; t < nr; t += blockDim.x) {
        double sd = 0.0;
        for (int w = 0; w < kWaves; ++w) sd += whs[w * nr + t];
        const float s = (float)sd;
        if (nsp > 1)
            k.hpart[((size_t)gsplit * k.geo.nwall + p) * nr + t] = s;
        else
            k.hist_out[(size_t)p * nr + t] = s * k.geo.att[t] * hs;
    }
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// Lane-serial backward drain: lane = one ray segment, kBSteps bins per round (the upstream
// gradient reads of a round are issued together), sums S_n = sum H pdf kap^n in registers.  A
// finished ray's closed-form result (dL/du0, dL/dv, dsigma, drho) is handed to the lane that owns
// its pair: finished lanes claim their pair lane with a forward permute (the highest claimant of a
// pair wins), each pair lane gathers its claimant's result with ds_bpermute and folds it into the
// Gaussian's register accumulators.  Losers keep their result and retry next round.  No LDS float
// atomics, no claim tables.
#ifndef NLOSGR_BSTEPS
#define NLOSGR_BSTEPS 24
#endif
constexpr int kBSteps = NLOSGR_BSTEPS;   // bins per lane per backward drain round
#ifndef NLOSGR_BSTEPS_NETF
// 20 since round 5 (spill-free with the SGPR wave index; C3 netf bwd 1684 -> 1618 ms; 24 spills 12 B)
#define NLOSGR_BSTEPS_NETF 20
#endif
#ifndef NLOSGR_BWD_WPE
#define NLOSGR_BWD_WPE 4   // backward: minimum waves per SIMD (4: <= 128 VGPRs)
#endif
#ifndef NLOSGR_BSTEPS_TAIL_SHR
// the shared-row layout's TAIL rounds (C5: bwd 941 / 855 / 824 ms per shard at 24 / 32 / 40 bins; 40 spills
// 64 B per lane in the wall-point loop, none in the drain)
#define NLOSGR_BSTEPS_TAIL_SHR 40
#endif
#ifndef NLOSGR_BSTEPS_NETF_TAIL
// netf TAIL rounds (round 5: exp-free cubic in pdf, D = drho / (sigma c dT); C3 netf bwd 1500 / 1478 / 1468 /
// 1485 ms at 24 / 28 / 32 / 36 bins; 32 spills 36 B per lane, in the wall-point loop, not in the drain)
#define NLOSGR_BSTEPS_NETF_TAIL 32
#endif
#ifndef NLOSGR_BPREFIX
#define NLOSGR_BPREFIX 1   // no-occlusion culled backward: moments by nested running sums (see bwd_kernel)
#endif
#ifndef NLOSGR_BSTEPS_TAIL
// (round 4's 40-bin rounds spilled 36 B per lane, reloaded and re-stored every wall point: ~1.2 GB of
// scratch writes per launch reached HBM.  The wave index read as an SGPR (readfirstlane) keeps the
// wave-derived LDS bases out of VGPRs and the kernel spill-free at 40; 32 bins cost ~30 ms per step;
// 48 / 56 bins: 767 / 776 vs 773 ms with 16 / 44 B of spills per lane — kept at 40, spill-free)
#define NLOSGR_BSTEPS_TAIL 40
#endif
// the staged gradient row is zero-padded by the longest round (no-occlusion TAIL rounds)
constexpr int kmax_i(int a, int b) { return a > b ? a : b; }
constexpr int kBPad = kmax_i(kmax_i(NLOSGR_BSTEPS_TAIL, kBSteps), kmax_i(NLOSGR_BSTEPS_NETF_TAIL, NLOSGR_BSTEPS_TAIL_SHR));
constexpr int kBwdSlots = 13;   // per-Gaussian backward partial: D[3], K~[3], 0[3] (shape_acc), dMu[3], dsigma
                                // (stride 32 in HBM)
constexpr int kShPart = 28;     // sh_kernel partial: dF[KM <= 25], dMu[3] (at KM), pad

// Two layouts.  Per-wave rows (default): each wave walks its own wall points and stages its own
// upstream-gradient row and angle tables.  Shared rows (bwd_shared, long rows): the workgroup's 4
// waves own 4 x 64 Gaussians and walk the same wall points; one double-buffered row + tables per
// workgroup (staged by all 256 threads one wall point ahead, one barrier per wall point), so the
// LDS no longer scales with 4 x nr (C5, nr = 2048: 56 KB -> 39 KB per workgroup, 2 -> 4 per CU).
struct BwdLayout {
    int wave_base, wave_stride, grow, tth, tph, rayq, pdat, red, total, buf_stride;
    __host__ __device__ BwdLayout(int nr, int nt, int np_, bool shared = false) {
        buf_stride = 0;
        if (shared) {
            grow = 0;                                 // buffer b at smem + b * buf_stride
            tth = al4(nr + kBPad);
            tph = tth + al4(2 * nt);
            buf_stride = tph + al4(2 * np_);
            wave_base = 2 * buf_stride;
            rayq = 0;                                 // per-wave region (relative to the wave's base)
            pdat = rayq + kRQ;
            wave_stride = al4(pdat + 64 * 16);
            red = 0;                                  // unused: waves own distinct Gaussians
            total = wave_base + kWaves * wave_stride;
            return;
        }
        wave_base = 0;
        grow = 0;                            // [nr + kBPad] upstream gradient x att x hscale, zero pad
        tth = al4(nr + kBPad);               // float2 [nt]
        tph = tth + al4(2 * nt);             // float2 [np]
        rayq = tph + al4(2 * np_);           // uint [kRQ] ring
        pdat = rayq + kRQ;                   // pair table, 4 planes [4][64] float4: A[0:4] | A[4:8] | A[8], u0 | r2, rho, sigma, r3
        wave_stride = al4(pdat + 64 * 16);
        red = wave_base;                     // final reduction reuses the wave regions
        total = wave_base + kWaves * wave_stride;
        const int need_red = wave_base + kWaves * 64 * kBwdSlots;
        if (need_red > total) total = need_red;
    }
};

// per-lane backward segment state
struct BRay {
    int pos, rem, slot, ij, kl, len;
    float kap, kap0, c0, c2, st;
    float S0, S1, S2;
    float zs[3], v[3], ts, w;            // ray geometry for the closed-form result
    float rho, sigma;
    float T, pre, dsig, drho;            // netf: transmittance, prefix of H out, accumulators (part A)
    float S0b, S1b, S2b, dsigb;          // netf: accumulators of part B (scaled by the ray's total at the end)
};

// The pair table is stored as four planes of 64 float4 (plane c = float4 c of every pair slot): a lane's
// ds_read_b128 of slot s starts at bank 4 (s mod 16), so the 16 lanes of a read group spread over the 16
// bank quads (a [64][16] row layout started every row at one of 4 banks: up to 16-way conflicts)
__device__ __forceinline__ void load_pdat(const float* pd, int slot, float* A, float* u0, float& w, float& rho,
                                          float& sigma) {
    const float4* q4 = reinterpret_cast<const float4*>(pd) + slot;
    const float4 a = q4[0], c = q4[64], e = q4[128], g = q4[192];
    A[0] = a.x; A[1] = a.y; A[2] = a.z; A[3] = a.w; A[4] = c.x; A[5] = c.y; A[6] = c.z; A[7] = c.w; A[8] = e.x;
    u0[0] = e.y; u0[1] = e.z; u0[2] = e.w;
    rho = g.y; sigma = g.z;
    w = sigma * rho;   // (= P.w of the pair setup, bit for bit)
}

// grow[k] = dL/dhist[p,k] att[k] hscale[p], zero-padded to nr + kBPad.  Rows of nr % 4 == 0
// are staged with 16-B loads issued together (one memory round trip per 1024 bins per lane).
// lane index the compiler cannot hoist: per-wall-point staging addresses are recomputed (a few
// VALU ops) instead of being kept live across the backward's wall-point loop (they spilled)
__device__ __forceinline__ int lane_opaque() {
    int l = lane_id();
    __asm__ __volatile__("" : "+v"(l));
    return l;
}

__device__ __forceinline__ void stage_grow(const float* grad, const float* att, float hs, int nr, float* grow) {
    const int lane = lane_opaque();
    if (grad && (nr & 3) == 0 && ((reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(att)) & 15) == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(grad);
        const float4* a4 = reinterpret_cast<const float4*>(att);
        const int n4 = nr >> 2;
        for (int t0 = lane; t0 < n4; t0 += 256) {
            float4 gv[4], av[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 64 * u;
                if (t < n4) { gv[u] = g4[t]; av[u] = a4[t]; }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 64 * u;
                if (t < n4)
                    reinterpret_cast<float4*>(grow)[t] =
                        make_float4(gv[u].x * av[u].x * hs, gv[u].y * av[u].y * hs, gv[u].z * av[u].z * hs,
                                    gv[u].w * av[u].w * hs);
            }
        }
    } else {
        for (int t = lane; t < nr; t += 64) grow[t] = grad ? grad[t] * att[t] * hs : 0.f;
    }
    for (int t = nr + lane; t < nr + kBPad; t += 64) grow[t] = 0.f;
}

// shared layout: the whole workgroup stages wall point p's row and tables into one buffer
__device__ __forceinline__ void stage_shared(const KArgs& k, int p, int nr, int nt, int np_, float* grow, float2* tth,
                                             float2* tph) {
    const int t0 = threadIdx.x;
    const float hs = k.geo.hscale[p];
    const float* grad = k.grad_hist ? k.grad_hist + (size_t)p * nr : nullptr;
    const float* att = k.geo.att;
    if (grad && (nr & 3) == 0 && ((reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(att)) & 15) == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(grad);
        const float4* a4 = reinterpret_cast<const float4*>(att);
        const int n4 = nr >> 2;
        for (int t = t0; t < n4; t += kBlock) {
            const float4 gv = g4[t], av = a4[t];
            reinterpret_cast<float4*>(grow)[t] =
                make_float4(gv.x * av.x * hs, gv.y * av.y * hs, gv.z * av.z * hs, gv.w * av.w * hs);
        }
    } else {
        for (int t = t0; t < nr; t += kBlock) grow[t] = grad ? grad[t] * att[t] * hs : 0.f;
    }
    for (int t = nr + t0; t < nr + kBPad; t += kBlock) grow[t] = 0.f;
    for (int t = t0; t < nt; t += kBlock)
        tth[t] = make_float2(k.geo.sin_theta[(size_t)p * nt + t], k.geo.cos_theta[(size_t)p * nt + t]);
    for (int t = t0; t < np_; t += kBlock)
        tph[t] = make_float2(k.geo.cos_phi[(size_t)p * np_ + t], k.geo.sin_phi[(size_t)p * np_ + t]);
}

template <int MODE, bool DENSE>
__device__ __forceinline__ bool bray_setup(const float* pd, float2 th, float2 ph, int slot, int i, int j, int nr,
                                           float mc2, float r0, float dr, float inv_dr, float f0log2, BRay& b) {
    float A[9], u0[3], w, rho, sigma;
    load_pdat(pd, slot, A, u0, w, rho, sigma);
    Ray R;
    if (!ray_setup<DENSE>(A, u0, th.x * ph.x, th.x * ph.y, th.y, mc2, r0, inv_dr, nr, R)) return false;
    b.pos = R.kl; b.kl = R.kl;
    b.len = b.rem = R.kh - R.kl + 1;
    b.slot = slot; b.ij = i | (j << 16);
    b.kap = b.kap0 = (float)R.kl - R.ks;
    b.c0 = -kHalfLog2e * R.m2min;
    b.c2 = -kHalfLog2e * R.a * dr * dr;
    b.st = th.x;
    b.S0 = b.S1 = b.S2 = 0.f;
    for (int r = 0; r < 3; ++r) { b.zs[r] = R.zs[r]; b.v[r] = R.v[r]; }
    b.ts = R.ts;
    b.w = w; b.rho = rho; b.sigma = sigma;
    if (MODE == NLOSGR_MODE_NETF) {
        b.T = fast_exp2((float)R.kl * f0log2);
        b.pre = b.dsig = b.drho = 0.f;
        b.S0b = b.S1b = b.S2b = b.dsigb = 0.f;
    }
    return true;
}

#ifndef NLOSGR_SHAPE_SENDER
#define NLOSGR_SHAPE_SENDER 1
#endif
constexpr bool kShapeSender = NLOSGR_SHAPE_SENDER;   // see rD / rK in bwd_kernel
#ifndef NLOSGR_NETF_CLOSED
#define NLOSGR_NETF_CLOSED 1
#endif
constexpr bool kNetfClosed = NLOSGR_NETF_CLOSED;     // netf TAIL backward: part B set at the ray start (bwd_kernel)

// TAIL (culled no-occlusion histogram backward at cutoff >= kTailCutoff): the drain reads the upstream
// row without the segment-end mask, see BV below

#ifdef NLOSGR_BCOUNT
// debug build (scripts/bwd_counts.py): loop iterations, drain rounds, active lanes, hand-off rounds,
// pending lanes, hand-offs done, refills, rays taken (per wave, summed), read by nlosgr_debug_bwd_counts
__device__ unsigned long long g_bdbg[8];
#define BDBG(i, v) bdbg[i] += (unsigned long long)(v)
#else
#define BDBG(i, v) ((void)0)
#endif

template <int PRESET, int MODE, bool DENSE, bool RAYS, bool CACHE, bool SHR, bool TAIL = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(NLOSGR_BWD_WPE, 8))) void bwd_kernel(KArgs k) {
#ifdef NLOSGR_BCOUNT
    unsigned long long bdbg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    // bins per drain round: netf keeps more per-ray state, so its rounds are shorter (no spill at 128 VGPRs)
    // (the no-occlusion TAIL rounds are longer: 32 bins measured 1137 vs 1170 ms at 24 on C3, and only
    // that variant stays spill-free at 32)
    constexpr int kRS = MODE == NLOSGR_MODE_NETF ? (TAIL && !RAYS && !DENSE ? NLOSGR_BSTEPS_NETF_TAIL : NLOSGR_BSTEPS_NETF)
                        : (MODE == NLOSGR_MODE_NOOCL && TAIL && !RAYS && !DENSE && !CACHE && !SHR) ? NLOSGR_BSTEPS_TAIL
                        : (MODE == NLOSGR_MODE_NOOCL && TAIL && !RAYS && !DENSE && !CACHE && SHR) ? NLOSGR_BSTEPS_TAIL_SHR : kBSteps;
    static_assert(kRS <= kBPad && kRS % 4 == 0, "the staged row is padded by kBPad bins; BV4 reads whole float4s");
    extern __shared__ __align__(16) float smem[];
    const int nr = k.geo.nr, nt = k.geo.nt, np_ = k.geo.np;
    constexpr bool shr = SHR;   // == (k.bshared != 0)
    const BwdLayout L(nr, nt, np_, shr);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();   // wave-uniform (SGPR)
    float* wb = smem + L.wave_base + wave * L.wave_stride;
    float* gbase = shr ? smem : wb;
    float* grow = gbase + L.grow;
    float2* tth = reinterpret_cast<float2*>(gbase + L.tth);
    float2* tph = reinterpret_cast<float2*>(gbase + L.tph);
    unsigned* rayq = reinterpret_cast<unsigned*>(wb + L.rayq);
    float* pdat = wb + L.pdat;

    const int gb = k.g_lo + blockIdx.x * (shr ? kNB * kWaves : kNB);
    const int gi = gb + (shr ? wave * kNB : 0) + lane;
    const bool active = gi < k.g_hi;
    const int split = blockIdx.y;
    const int per = (k.pnw + k.nsplit - 1) / k.nsplit;
    const int pbeg = k.pb0 + split * per, pend = min(k.pb0 + k.pnw, pbeg + per);
    const int deg = k.g.sh_degree;
    const int K = (deg + 1) * (deg + 1);
    const float mc2 = k.opt.cutoff * k.opt.cutoff;
    const float r0 = k.geo.r[0];
    const float dr = nr > 1 ? (k.geo.r[nr - 1] - r0) / (float)(nr - 1) : 0.f;
    const float inv_dr = dr > 0.f ? 1.0f / dr : 0.f;
    const float cdt = k.opt.c_deltaT;
    const bool small_x = cdt <= kSmallX;   // netf: exp-free transmittance factor (om_exp_small)
    const float f0log2 = log2f(1.0f + 1e-7f);
    const float rscale = k.opt.ray_scale;

    // shape accumulators (shape_acc: D = diag of dA A^T, K~ = its rotational part), dL/dmu, dL/dsigma
    float sD[3] = {0.f, 0.f, 0.f}, sK[3] = {0.f, 0.f, 0.f}, dMu[3], dSig = 0.f;
    dMu[0] = dMu[1] = dMu[2] = 0.f;
    // this lane's Gaussian: record and feature row are re-read per wall point (L1/L2 hits) rather
    // than held in registers across the split (VGPR budget)
    // (mu too: a register copy across the wall-point loop spilled at the longer netf rounds)
    const float* feat = k.g.features + (size_t)(active ? gi : 0) * k.g.k_feat;

    if (shr && pbeg < pend) stage_shared(k, pbeg, nr, nt, np_, grow, tth, tph);
    int it = 0;
    for (int p = pbeg + (shr ? 0 : wave); p < pend; p += (shr ? 1 : kWaves), ++it) {
        // stage this wall point's upstream gradient row and tables (wave-private), or (shared) make
        // the buffer staged one wall point ahead current and stage the next one into the other
        const float hs = k.geo.hscale[p];
        wave_sync();
        if (shr) {
            __syncthreads();   // buffer it & 1 complete; every wave is done with wall point p - 1
            float* bnext = smem + ((it + 1) & 1) * L.buf_stride;
            if (p + 1 < pend)
                stage_shared(k, p + 1, nr, nt, np_, bnext + L.grow, reinterpret_cast<float2*>(bnext + L.tth),
                             reinterpret_cast<float2*>(bnext + L.tph));
            float* bcur = smem + (it & 1) * L.buf_stride;
            grow = bcur + L.grow;
            tth = reinterpret_cast<float2*>(bcur + L.tth);
            tph = reinterpret_cast<float2*>(bcur + L.tph);
        } else {
            stage_grow(k.grad_hist ? k.grad_hist + (size_t)p * nr : nullptr, k.geo.att, hs, nr, grow);
            const int ln = lane_opaque();
            for (int t = ln; t < nt; t += 64)
                tth[t] = make_float2(k.geo.sin_theta[(size_t)p * nt + t], k.geo.cos_theta[(size_t)p * nt + t]);
            for (int t = ln; t < np_; t += 64)
                tph[t] = make_float2(k.geo.cos_phi[(size_t)p * np_ + t], k.geo.sin_phi[(size_t)p * np_ + t]);
        }
        const float px = k.geo.wall[3 * p], py = k.geo.wall[3 * p + 1], pz = k.geo.wall[3 * p + 2];
        // per-pair row offset, recomputed per wall point (not hoisted as per-lane 64-bit pointers)
        int gio = gi;
        __asm__ __volatile__("" : "+v"(gio));
        const size_t o = (size_t)p * k.g.ng + gio;
        // pair setup (lane = Gaussian gi at wall point p); the ray pass reads the pair table
        bool more = false;
        float M[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int i0 = 0, i1 = -1, j0 = 0, j1 = -1;
        float wpair = 0.f;
        unsigned bx = 0u;
        if (active) {
            Pair P;
            float mu[3];
            load_rec(k.recs[gi], P, mu);
            if (CACHE) bx = k.cbox[o];
            if (CACHE && bx != 0u) {
                // cached pair: u0 and the forward's albedo; no SH evaluation, no footprint (the
                // recorded cells replace the quadric walk)
                P.q[0] = px - mu[0]; P.q[1] = py - mu[1]; P.q[2] = pz - mu[2];
                for (int r = 0; r < 3; ++r)
                    P.u0[r] = P.A[3 * r] * P.q[0] + P.A[3 * r + 1] * P.q[1] + P.A[3 * r + 2] * P.q[2];
                P.rho = k.crho[o];
                P.w = P.sigma * P.rho;
                P.i0 = P.j0 = 0; P.i1 = P.j1 = 0;
                for (int t = 0; t < 6; ++t) P.M[t] = 0.f;
            } else {
                pair_setup<PRESET, DENSE>(k, feat, mu, px, py, pz, k.geo.grid_lin + 4 * (size_t)p, mc2, P);
            }
            more = (P.w > 0.f) && P.i0 <= P.i1 && P.j0 <= P.j1 && !(k.opt.flags & 2);  // flags 2: setup only
            for (int t = 0; t < 6; ++t) M[t] = P.M[t];
            i0 = P.i0; i1 = P.i1; j0 = P.j0; j1 = P.j1;
            wpair = P.w;
            float4* d4 = reinterpret_cast<float4*>(pdat) + lane;
            d4[0] = make_float4(P.A[0], P.A[1], P.A[2], P.A[3]);
            d4[64] = make_float4(P.A[4], P.A[5], P.A[6], P.A[7]);
            d4[128] = make_float4(P.A[8], P.u0[0], P.u0[1], P.u0[2]);
            float r2, r3;
            scale_ratios(P.A, r2, r3);
            d4[192] = make_float4(r2, P.rho, P.sigma, r3);
        }
        // ray cache of the forward: cached pairs walk their recorded cells instead of enumerating
        unsigned long long cbits0 = 0ull, cbits1 = 0ull;
        int ci0 = 0, cj0 = 0, cw = 1;
        float rcw = 1.f;
        if (CACHE && active) {
            if (bx != 0u) {
                const ulonglong2 cm = k.cmask[o];
                cbits0 = more ? cm.x : 0ull;
                cbits1 = more ? cm.y : 0ull;
                ci0 = bx & 0xFFF; cj0 = (bx >> 12) & 0xFFF; cw = bx >> 24;
                rcw = 1.0f / (float)cw;
                more = false;
            }
        }
        const float* gray = RAYS && k.grad_ray ? k.grad_ray + (size_t)p * nt * np_ * nr : nullptr;
        wave_sync();
        int ci = i0, cj = j0, qhead = 0, qcount = 0;
        bool act = false, pend = false;
        float dU0p[3] = {0.f, 0.f, 0.f}, drho_pair = 0.f, s0_pair = 0.f;
        BRay b;
        b.pos = 0; b.rem = 0; b.slot = lane; b.ij = 0; b.kl = 0; b.len = 0;
        b.kap = b.kap0 = b.c0 = b.c2 = b.st = 0.f;
        b.S0 = b.S1 = b.S2 = 0.f;
        b.zs[0] = b.zs[1] = b.zs[2] = b.v[0] = b.v[1] = b.v[2] = b.ts = b.w = 0.f;
        b.rho = b.sigma = 0.f;
        b.T = b.pre = b.dsig = b.drho = 0.f;
        b.S0b = b.S1b = b.S2b = b.dsigb = 0.f;
        // pending result of a finished ray: dL/du0, dL/dv, dsigma, drho
        // kShapeSender: the ray's dL/dA contribution dL/dv d^T goes over as shape_acc's (D, K~), formed at the
        // ray's end (rD, rK); otherwise dL/dv and v go over and the pair lane forms it per hand-off round
        float rU[3] = {0.f, 0.f, 0.f}, rD[3] = {0.f, 0.f, 0.f}, rK[3] = {0.f, 0.f, 0.f}, rSig = 0.f, rRho = 0.f;
        while (true) {
            if (CACHE && qcount < 64 && __builtin_amdgcn_ballot_w64((cbits0 | cbits1) != 0ull)) {
                wave_sync();
                enumerate_cached(cbits0, cbits1, ci0, cj0, cw, rcw, rayq, qhead, qcount);
                wave_sync();
            }
            if (qcount < 64 && __builtin_amdgcn_ballot_w64(more)) {
                wave_sync();
                enumerate_box<DENSE>(M, i1, j0, j1, more, ci, cj, tth, tph, nt - 1, rayq, qhead, qcount);
                wave_sync();
            }
            const bool anymore = __builtin_amdgcn_ballot_w64(more || (CACHE && (cbits0 | cbits1) != 0ull)) != 0;
            // a lane whose finished result still waits for its hand-off takes no new ray
            const unsigned long long idle = __builtin_amdgcn_ballot_w64(!act && !pend);
            const int nidle = __popcll(idle);
            if (qcount > 0 && (nidle >= kBRefill || !anymore)) {
                const int r = lanes_below(idle);
                const bool take = !act && !pend && r < qcount;
                if (take && !(k.opt.flags & 1)) {                  // flags 1: enumerate only
                    const unsigned e = rayq[(qhead + r) & (kRQ - 1)];
                    const int slot = e & 0xFF, i = (e >> 8) & 0xFFF, j = e >> 20;
                    act = bray_setup<MODE, DENSE>(pdat, tth[i], tph[j], slot, i, j, nr, mc2, r0, dr,
                                                  inv_dr, f0log2, b) && !(k.opt.flags & 4);  // flags 4: no bins
                    if (MODE == NLOSGR_MODE_NETF && TAIL) b.T *= b.st;   // sin(theta) rides on T (BV rows)
                    if (MODE == NLOSGR_MODE_NETF && TAIL && !DENSE && kNetfClosed && act) {
                        // part B's sums are a_c sigma sum_j pdf_j (1, kap_j, kap_j^2) over the ray's bins, which the
                        // TAIL rounds cover to past 5 sigma on both sides: they are set here once instead of 3 VALU
                        // per bin.  A ray at least one bin wide (sigma_b^2 = 1 / (a dr^2) >= 1) whose Gaussian lies
                        // inside the histogram by 6 sigma_b on both sides: its own moments 2^c0 sqrt(2 pi) sigma_b
                        // (1, 0, sigma_b^2) (Poisson summation: relative error <= exp(-2 pi^2 sigma_b^2) < 3e-9, plus
                        // the tails past 5 sigma the rounds leave out, < 3e-7 of the ray's sum); any other (narrow, or
                        // cut by the first or last bin): its support bins [kl, kh] summed here
                        const float sb2 = kHalfLog2e * frcp(-b.c2);
                        const float ksb = (float)b.kl - b.kap0;   // the closest approach, in bins
                        const float w6 = 6.0f * __builtin_amdgcn_sqrtf(sb2);
                        float g0 = 0.f, g1 = 0.f, g2 = 0.f;
                        if (sb2 >= 1.0f && ksb - w6 >= 0.f && ksb + w6 <= (float)(nr - 1)) {
                            g0 = fast_exp2(b.c0) * (2.50662827463f * __builtin_amdgcn_sqrtf(sb2));
                            g2 = g0 * sb2;
                        } else {
                            for (int jb = b.kl; jb < b.kl + b.len; ++jb) {
                                const float kj = b.kap0 + (float)(jb - b.kl);
                                const float pj = fast_exp2(fmaf(b.c2, kj * kj, b.c0));
                                g0 += pj;
                                g1 = fmaf(pj, kj, g1);
                                g2 = fmaf(pj * kj, kj, g2);
                            }
                        }
                        const float acl = -cdt / (1.0f + 1e-7f);
                        b.S0b = b.sigma * acl * g0;
                        b.S1b = b.sigma * acl * g1;
                        b.S2b = b.sigma * acl * g2;
                        b.dsigb = acl * g0;
                    }
                }
                const int ntake = min(nidle, qcount);
                BDBG(6, 1); BDBG(7, ntake);
                qhead = (qhead + ntake) & (kRQ - 1);
                qcount -= ntake;
            }
            const bool anyact = __builtin_amdgcn_ballot_w64(act) != 0;
            const bool anypend = __builtin_amdgcn_ballot_w64(pend) != 0;
            if (!anyact && !anypend) {
                if (!anymore && qcount == 0) break;
                continue;
            }
            BDBG(0, 1);
            if (anyact) { BDBG(1, 1); BDBG(2, __popcll(__builtin_amdgcn_ballot_w64(act))); }
            if (anyact) {
                const int remw = act ? b.rem : 0;
                // BV: the round starts at the even bin at or below pos (float2 row reads, half the LDS
                // instructions); slot j is bin (pos & ~1) + j, in the segment iff o <= j < remw + o
                constexpr bool BV = (MODE == NLOSGR_MODE_NOOCL || (MODE == NLOSGR_MODE_NETF && TAIL)) && !RAYS && !DENSE;
                // BV4 (no-occlusion TAIL): the round starts at the bin at or below pos that is a multiple of
                // 4 and reads the row as float4 (ds_read_b128: 16-lane groups over 16 bank quads conflict
                // less per bin than 32-lane groups over 32 bank pairs, and half the instructions)
                // (netf TAIL measured 20 ms slower with float4 reads: C3 netf bwd 1537 -> 1557 ms)
                constexpr bool BV4 = MODE == NLOSGR_MODE_NOOCL && TAIL && !RAYS && !DENSE;
                constexpr int BVW = BV4 ? 4 : 2;
                const int o = BV && act ? (b.pos & (BVW - 1)) : 0;
                const float* gr = grow + (act ? b.pos - o : 0);
                const float* gw = RAYS && gray ? gray + (size_t)((b.ij & 0xFFFF) * np_ + (b.ij >> 16)) * nr + b.pos
                                               : nullptr;
                float Hs[kRS];
                if (BV4) {
                    // as below, with slots 0..o-1 before pos masked (o <= 3)
                    const float4* g4 = reinterpret_cast<const float4*>(gr);
#pragma unroll
                    for (int m = 0; m < kRS; m += 4) {
                        const float4 h = g4[m / 4];
                        Hs[m] = (m == 0 && o > 0) ? 0.f : h.x;
                        Hs[m + 1] = (m == 0 && o > 1) ? 0.f : h.y;
                        Hs[m + 2] = (m == 0 && o > 2) ? 0.f : h.z;
                        Hs[m + 3] = h.w;
                    }
                } else if (BV && TAIL) {
                    // no end mask: a segment's last round also weighs the bins past its end (up to
                    // kRS - 1 of them) with their exact pdf, < exp(-m_c^2 / 2) of the Gaussian's peak
                    // (<= 3.7e-6 at m_c >= kTailCutoff: the support is a superset of the forward's, closer
                    // to the dense reference; idle and blocked lanes are zeroed through their pdf seed
                    // below).  Slot 0 before pos (o = 1) stays masked: the recurrence starts at pos.
                    const float2* g2 = reinterpret_cast<const float2*>(gr);
#pragma unroll
                    for (int m = 0; m < kRS; m += 2) {
                        const float2 h = g2[m / 2];
                        Hs[m] = (m == 0 && o) ? 0.f : h.x;
                        Hs[m + 1] = h.y;
                    }
                } else if (BV) {
                    const int lim = remw + o;
                    const float2* g2 = reinterpret_cast<const float2*>(gr);
#pragma unroll
                    for (int m = 0; m < kRS; m += 2) {
                        const float2 h = g2[m / 2];
                        Hs[m] = (m >= o && m < lim) ? h.x : 0.f;
                        Hs[m + 1] = (m + 1 < lim) ? h.y : 0.f;
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < kRS; ++m) {
                        float H = gr[m];
                        if (RAYS || MODE == NLOSGR_MODE_NETF) H *= b.st;
                        if (RAYS && gw && m < remw) H += gw[m] * rscale;
                        Hs[m] = m < remw ? H : 0.f;
                    }
                }
                float kap = b.kap;
                if (MODE == NLOSGR_MODE_NOOCL) {
                    float S0 = b.S0, S1 = b.S1, S2 = b.S2;
                    if (!DENSE) {
                        // exp2 recurrence (kRecurrence) and moments about the round's first bin:
                        // U_n = sum_m hp m^n, then S_n += sum_m hp (kap + m)^n
                        float pdf = fast_exp2(fmaf(b.c2, kap * kap, b.c0));
                        // BV reads the row unmasked: idle lanes and blocked ones (finished, rem <= 0, waiting
                        // for their hand-off) contribute through a zero seed
                        if (BV && TAIL && !(act && b.rem > 0)) pdf = 0.f;
                        float q = fast_exp2(b.c2 * fmaf(2.f, kap, 1.f));
                        const float cc = fast_exp2(2.f * b.c2);
#if NLOSGR_BPREFIX
                        // three nested running sums (one fma, two adds per bin): with w = kRS - m,
                        // A = sum hp, B = sum hp w, C = sum hp w (w + 1) / 2, hp = H pdf; then about
                        // K = kap at slot kRS: sum hp (K - w)^n for n = 0, 1, 2 (w^2 sums to 2C - B)
                        float A = 0.f, B = 0.f, C = 0.f;
#pragma unroll
                        for (int m = 0; m < kRS; ++m) {
                            A = fmaf(Hs[m], pdf, A);
                            B += A;
                            C += B;
                            if (BV && m < BVW - 1) {   // the recurrence starts at pos (slot o)
                                pdf = m < o ? pdf : pdf * q;
                                q = m < o ? q : q * cc;
                            } else {
                                pdf *= q;
                                q *= cc;
                            }
                        }
                        const float K = kap - (float)o + (float)kRS;
                        S0 += A;
                        S1 += fmaf(K, A, -B);
                        S2 += fmaf(K, fmaf(K, A, -2.f * B), fmaf(2.f, C, -B));
#else
                        float U0 = 0.f, U1 = 0.f, U2 = 0.f;
#pragma unroll
                        for (int m = 0; m < kRS; ++m) {
                            const float hp = Hs[m] * pdf;
                            U0 += hp;
                            U1 = fmaf(hp, (float)m, U1);
                            U2 = fmaf(hp, (float)(m * m), U2);
                            if (BV && m < BVW - 1) {   // the recurrence starts at pos (slot o)
                                pdf = m < o ? pdf : pdf * q;
                                q = m < o ? q : q * cc;
                            } else {
                                pdf *= q;
                                q *= cc;
                            }
                        }
                        const float kb = kap - (float)o;   // kap at slot 0
                        S0 += U0;
                        S1 += fmaf(kb, U0, U1);
                        S2 += fmaf(kb, fmaf(kb, U0, 2.f * U1), U2);
#endif
                        kap += (float)(kRS - o);
                    } else
#pragma unroll
                    for (int m = 0; m < kRS; ++m) {
                        const float hp = Hs[m] * fast_exp2(fmaf(b.c2, kap * kap, b.c0));
                        const float t1 = hp * kap;
                        S0 += hp; S1 += t1; S2 = fmaf(t1, kap, S2);
                        kap += 1.f;
                    }
                    b.S0 = S0; b.S1 = S1; b.S2 = S2;
                } else {
                    // dL/dD_j = c rho H_j T_j + a_j (E - P_j),  a_j = f'_j / f_j = -c dT e_j / f_j, P_j = the
                    // prefix sum of H_k out_k through bin j and E its total over the ray.  One pass: every
                    // weighted sum sum_j dL/dD_j w_j splits into part A = sum_j (c rho H_j T_j - P_j a_j) w_j and
                    // part B = sum_j a_j w_j, combined as A + E B once the ray is done (E = P at the end).
                    float T = b.T, pre = b.pre;
                    float S0 = b.S0, S1 = b.S1, S2 = b.S2, dsig = b.dsig, drho = b.drho;
                    float S0b = b.S0b, S1b = b.S1b, S2b = b.S2b, dsigb = b.dsigb;
                    const float kE = -cdt * (2.f * kHalfLog2e) * b.sigma, ncdt = -cdt, crho = cdt * b.rho;
                    // culled: pdf by the exp2 recurrence (kRecurrence), re-seeded per round
                    float cur = 0.f, rq = 0.f, rcc = 0.f;
                    // TAIL: the recurrence starts at slot 0 = bin pos - o; inactive lanes get a zero seed
                    const float kseed = TAIL ? kap - (float)o : kap;
                    if (!DENSE) {
                        cur = fast_exp2(fmaf(b.c2, kseed * kseed, b.c0));
                        rq = fast_exp2(b.c2 * fmaf(2.f, kseed, 1.f));
                        rcc = fast_exp2(2.f * b.c2);
                        if (TAIL && !(act && b.rem > 0)) cur = 0.f;
                    }
                    if (!DENSE && (small_x || TAIL)) {   // (netf TAIL is launched only when small_x)
                        // c dT <= 1/64: x = sigma pdf c dT <= c dT, so exp(-x) = 1 - om_exp_small(x) (no
                        // exp) and a_j = -c dT e_j / (e_j + 1e-7) = -c dT / (1 + 1e-7 / e_j) is the constant
                        // a_c = -c dT / (1 + 1e-7) to 1e-7 x relative (no rcp): part B's sums become
                        // a_c sum pdf (1, m, m^2) (moments about the round's first bin, like U_n above)
                        const float sx = cdt * b.sigma;
                        const float ac = ncdt / (1.0f + 1e-7f);
                        // exp(-x) + 1e-7 for x = sx pdf <= 1/64 as a cubic in pdf (the x^4 / 24 term, <= 2.5e-9,
                        // is dropped; the forward's factor, kTf0 = 1 + 1e-7 in float)
                        const float e1 = -sx, e2 = 0.5f * sx * sx, e3 = (-1.0f / 6.0f) * sx * sx * sx;
                        // the prefix P_j = rho sum_{k<=j} H_k T_k x_k = rho sx D_j with D_j = sum_{k<=j} H_k T_k pdf_k
                        // (this path keeps D in b.drho; rho is the pair's), so part A's weight is
                        // c rho H_j T_j - P_j a_c = crho (HT + kk D) with kk = -a_c sigma; sum_j c1_j pdf_j
                        // (dsigma's part A) is crho UA0, summed per round below
                        const float kk = -ac * b.sigma;
                        // part A's moments by nested running sums (as the no-occlusion drain): UA0 = sum hA,
                        // UA1 = sum hA w, UA2 = sum hA w (w + 1) / 2 with w = kRS - m; part B's directly
                        float UA0 = 0.f, UA1 = 0.f, UA2 = 0.f, UB0 = 0.f, UB1 = 0.f, UB2 = 0.f;
                        constexpr bool UB = !(TAIL && kNetfClosed);   // part B per bin (else set at the ray's start)
#pragma unroll
                        for (int m = 0; m < kRS; ++m) {
                            // TAIL: no segment-end mask (the bins past the end carry the Gaussian's exact
                            // tail, as in the no-occlusion drains); only slot 0 before pos (o = 1) in a
                            // segment's first round is inactive.  sin(theta) is folded into T (bray start).
                            const bool in = TAIL ? !(m == 0 && o) : m < remw;
                            const float pdf = cur;
                            cur *= rq;
                            rq *= rcc;
                            const float f = fmaf(pdf, fmaf(pdf, fmaf(pdf, e3, e2), e1), kTf0);
                            const float HT = Hs[m] * T;
                            drho = fmaf(HT, pdf, drho);               // D
                            const float c1 = in ? fmaf(kk, drho, HT) : 0.f;
                            UA0 = fmaf(c1, pdf, UA0);                 // x crho sigma at the end
                            UA1 += UA0;
                            UA2 += UA1;
                            if (UB) {
                                const float pin = in ? pdf : 0.f;
                                UB0 += pin;
                                UB1 = fmaf(pin, (float)m, UB1);
                                UB2 = fmaf(pin, (float)(m * m), UB2);
                            }
                            T *= in ? f : 1.f;
                        }
                        dsig = fmaf(crho, UA0, dsig);
                        pre = b.rho * sx * drho;
                        // S_n += sum h (kb + m)^n, kb = the round's first bin offset
                        const float kb = kseed;
                        const float sg = b.sigma * crho;
                        const float sgb = b.sigma * ac;
                        const float KA = kb + (float)kRS;   // kap at slot kRS
                        S0 = fmaf(sg, UA0, S0);
                        S1 = fmaf(sg, fmaf(KA, UA0, -UA1), S1);
                        S2 = fmaf(sg, fmaf(KA, fmaf(KA, UA0, -2.f * UA1), fmaf(2.f, UA2, -UA1)), S2);
                        S0b = fmaf(sgb, UB0, S0b);
                        S1b = fmaf(sgb, fmaf(kb, UB0, UB1), S1b);
                        S2b = fmaf(sgb, fmaf(kb, fmaf(kb, UB0, 2.f * UB1), UB2), S2b);
                        dsigb = fmaf(ac, UB0, dsigb);
                        kap += (float)(kRS - o);
                    } else {
#pragma unroll
                    for (int m = 0; m < kRS; ++m) {
                        const bool in = m < remw;
                        float pdf;
                        if (DENSE) {
                            pdf = fast_exp2(fmaf(b.c2, kap * kap, b.c0));
                        } else {
                            pdf = cur;
                            cur *= rq;
                            rq *= rcc;
                        }
                        // per-ray constants folded: sp = sigma pdf, exp(-sp c dT) = exp2(pdf kE)
                        const float sp = b.sigma * pdf;
                        const float H = Hs[m];
                        const float ee = fast_exp2(pdf * kE);
                        const float f = ee + 1e-7f;
                        const float HT = H * T;
                        const float hdt = HT * (cdt * sp);
                        drho += hdt;
                        pre = fmaf(b.rho, hdt, pre);
                        const float a = in ? (ee * ncdt) * frcp(f) : 0.f;
                        const float c1 = in ? fmaf(-pre, a, crho * HT) : 0.f;
                        const float hA = c1 * sp, hB = a * sp;
                        dsig = fmaf(c1, pdf, dsig);
                        dsigb = fmaf(a, pdf, dsigb);
                        const float tA = hA * kap, tB = hB * kap;
                        S0 += hA; S1 += tA; S2 = fmaf(tA, kap, S2);
                        S0b += hB; S1b += tB; S2b = fmaf(tB, kap, S2b);
                        T *= in ? f : 1.f;
                        kap += 1.f;
                    }
                    }
                    b.T = T; b.pre = pre;
                    b.S0b = S0b; b.S1b = S1b; b.S2b = S2b; b.dsigb = dsigb;
                    b.S0 = S0; b.S1 = S1; b.S2 = S2; b.dsig = dsig; b.drho = drho;
                }
                if (act) {
                    if (b.rem > 0) {   // (a blocked lane, rem <= 0, added zeros and stays put)
                        b.kap = kap;
                        b.pos += kRS - o;
                        b.rem -= kRS - o;
                    }
                    if (b.rem <= 0 && !pend) {
                        // pdf = exp(-|z|^2/2), z = z* + dl v:  dL/du0 = -sum P z,  dL/dv = -sum P dl z
                        float S0 = b.S0, S1 = b.S1, S2 = b.S2;
                        if (MODE == NLOSGR_MODE_NETF) {   // A + E B, E = the ray's total (its final prefix)
                            S0 = fmaf(b.pre, b.S0b, S0);
                            S1 = fmaf(b.pre, b.S1b, S1);
                            S2 = fmaf(b.pre, b.S2b, S2);
                        }
                        S1 = S1 * dr;
                        S2 = S2 * dr * dr;
                        if (MODE == NLOSGR_MODE_NOOCL) {
                            if (!RAYS) { S0 *= b.st; S1 *= b.st; S2 *= b.st; }
                            // no-occlusion: dsigma = S0 rho, drho = S0 sigma; the pair lane applies its own
                            // rho and sigma to the summed S0 (one value handed over instead of two)
                            rSig = S0;
                            rRho = 0.f;
                            S0 *= b.w; S1 *= b.w; S2 *= b.w;
                        } else {
                            rSig = fmaf(b.pre, b.dsigb, b.dsig);
                            // (the exp-free culled drain keeps D = drho / (sigma c dT) in b.drho)
                            rRho = !DENSE && (small_x || TAIL) ? b.drho * (cdt * b.sigma) : b.drho;
                        }
                        float rV[3];
                        for (int r = 0; r < 3; ++r) {
                            const float zv = S0 * b.zs[r] + S1 * b.v[r];
                            rU[r] = -zv;
                            rV[r] = -(b.ts * zv + S1 * b.zs[r] + S2 * b.v[r]);
                        }
                        if (kShapeSender) {
                            // dL/dA += dL/dv d^T, in whitened form shape_acc(dL/dv, v = A d) with the pair's
                            // scale ratios (pair table plane 3), formed once here rather than per hand-off round
                            const float4 rr = reinterpret_cast<const float4*>(pdat)[192 + b.slot];   // r2, rho, sigma, r3
                            rD[0] = rD[1] = rD[2] = rK[0] = rK[1] = rK[2] = 0.f;
                            shape_acc(rV, b.v, rr.x, rr.w, rD, rK);
                        } else {
                            rD[0] = rV[0]; rD[1] = rV[1]; rD[2] = rV[2];   // (dL/dv; v stays in b.v)
                        }
                        act = false;
                        pend = !(k.opt.flags & 32);   // flags 32 (diagnostics): drop results, no hand-off
                    }
                }
            }
            const unsigned long long pmask = __builtin_amdgcn_ballot_w64(pend);
            if (pmask) {
                // hand finished rays to their pair lanes: per pair and round one claimant, its result
                // fetched by the pair lane with bpermute.  The claim is a forward permute (ds_permute_b32,
                // no LDS memory, no fences): every pending lane sends lane + 1 to its pair lane, and of
                // several senders to one lane the highest lane's value arrives (lanes nobody writes
                // receive 0; measured on gfx950, scripts/permute_probe.hip).  Every lane that must
                // receive also sends, so the lanes without a result park a 0 on lane 0 in one permute and
                // on lane 1 in a second; lane 0 reads the second, every other lane the first.
                const int pv = pend ? lane + 1 : 0;
                const int w1 = __builtin_amdgcn_ds_permute((pend ? b.slot : 0) << 2, pv);
                const int w2 = __builtin_amdgcn_ds_permute((pend ? b.slot : 1) << 2, pv);
                const int wcl = lane == 0 ? w2 : w1;
                const bool got = wcl != 0;
                const int src = got ? wcl - 1 : lane;
                // (all lanes execute the bpermute: a source lane inactive in EXEC reads as 0)
                const int wpair = __builtin_amdgcn_ds_bpermute(b.slot << 2, wcl);
                const bool won = pend && wpair == lane + 1;
                const float gm = got ? 1.f : 0.f;
                float gU[3];
                // every lane must execute the bpermute: it cannot read lanes that are inactive in EXEC
                if (kShapeSender) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        gU[c] = gm * __shfl(rU[c], src);
                        sD[c] += gm * __shfl(rD[c], src);
                        sK[c] += gm * __shfl(rK[c], src);
                    }
                } else {
                    float gV[3], gW[3];
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        gU[c] = gm * __shfl(rU[c], src);
                        gV[c] = gm * __shfl(rD[c], src);
                        gW[c] = __shfl(b.v[c], src);
                    }
                    const float4 rr = reinterpret_cast<const float4*>(pdat)[192 + lane];   // r2, rho, sigma, r3
                    shape_acc(gV, gW, rr.x, rr.w, sD, sK);
                }
                const float gSig = gm * __shfl(rSig, src);
                const float gRho = MODE == NLOSGR_MODE_NOOCL ? 0.f : gm * __shfl(rRho, src);
                for (int r = 0; r < 3; ++r) dU0p[r] += gU[r];
                if (MODE == NLOSGR_MODE_NOOCL) {
                    s0_pair += gSig;
                } else {
                    dSig += gSig;
                    drho_pair += gRho;
                }
                BDBG(3, 1); BDBG(4, __popcll(pmask)); BDBG(5, __popcll(__builtin_amdgcn_ballot_w64(won)));
                if (won) pend = false;
            }
        }
        // chain of this wall point's pair (Gaussian gi, wall point p) through u0 = A (p - mu); the
        // view-direction chain through rho (SH basis, d_features and its d_mu share) runs in
        // sh_kernel from the stored dL/drho, which keeps 16 feature accumulators out of this kernel
        if (MODE == NLOSGR_MODE_NOOCL && active) {
            const float4 wrs = reinterpret_cast<const float4*>(pdat)[192 + lane];   // w, rho, sigma
            dSig += s0_pair * wrs.y;
            drho_pair = s0_pair * wrs.z;
        }
        if (active && wpair > 0.f) {
            // dL/dA += dL/du0 (p - mu)^T, as shape_acc(dL/du0, u0) with u0 = A (p - mu) from the pair table
            const float4* d4 = reinterpret_cast<const float4*>(pdat) + lane;
            const float4 a = d4[0], c = d4[64], e = d4[128], rr = d4[192];
            const float A[9] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w, e.x};
            const float u0[3] = {e.y, e.z, e.w};
            shape_acc(dU0p, u0, rr.x, rr.w, sD, sK);
            for (int cc = 0; cc < 3; ++cc) dMu[cc] -= A[cc] * dU0p[0] + A[3 + cc] * dU0p[1] + A[6 + cc] * dU0p[2];
        }
        if (active) k.drho[(size_t)(p - k.pb0) * k.g.ng + gio] = (wpair > 0.f && !(k.opt.flags & 64)) ? drho_pair : 0.f;
    }
#ifdef NLOSGR_BCOUNT
    if (lane == 0)
        for (int c = 0; c < 8; ++c) atomicAdd(&g_bdbg[c], bdbg[c]);
#endif
    if (shr) {   // shared layout: every wave owns its Gaussians for the whole split
        if (active) {
            // (rows of this split belong to this workgroup only; the first batch overwrites whatever the
            // workspace held, later batches add)
            float* dst = k.partial + ((size_t)split * k.g.ng + gi) * 32;
            float v[kBwdSlots];
            for (int t = 0; t < 3; ++t) { v[t] = sD[t]; v[3 + t] = sK[t]; v[6 + t] = 0.f; }
            v[9] = dMu[0]; v[10] = dMu[1]; v[11] = dMu[2]; v[12] = dSig;
            if (k.accum)
                for (int t = 0; t < kBwdSlots; ++t) v[t] += dst[t];
            for (int t = 0; t < kBwdSlots; ++t) dst[t] = v[t];
        }
        return;
    }
    // fixed-order combination of the 4 waves' accumulators -> partial slab
    __syncthreads();
    float* red = smem + L.red;
    {
        float* dst = red + (wave * 64 + lane) * kBwdSlots;
        for (int t = 0; t < 3; ++t) { dst[t] = sD[t]; dst[3 + t] = sK[t]; dst[6 + t] = 0.f; }
        dst[9] = dMu[0]; dst[10] = dMu[1]; dst[11] = dMu[2];
        dst[12] = dSig;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < kNB * kBwdSlots; t += blockDim.x) {
        const int g = t / kBwdSlots, c = t - g * kBwdSlots;
        if (gb + g >= k.g_hi) continue;
        float s = 0.f;
        for (int w = 0; w < kWaves; ++w) s += red[(w * 64 + g) * kBwdSlots + c];
        float* dst = k.partial + ((size_t)split * k.g.ng + gb + g) * 32 + c;
        *dst = k.accum ? *dst + s : s;
    }
}

// ------------------------------------------------------------------------------------------
// sh_kernel: the view-direction chain of every pair from the backward's dL/drho (fixed wall-point
// order within each of nsh splits): d_features += drho Y(dir), d_mu += drho (dY/ddir . f) ddir/dmu,
// dir = view direction of mu - p (preset convention; nlos_helpers / cuda_utils.cuh semantics as in
// the forward's pair_setup).  One lane per Gaussian; drho rows [P][ng] are read coalesced.
// ------------------------------------------------------------------------------------------
// KM: coefficient registers (16 up to degree 3, 25 for degree 4); partial rows of kShPart floats
template <int PRESET, int KM>
__global__ __launch_bounds__(kBlock) void sh_kernel(KArgs k) {
    const int gi = k.g_lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= k.g_hi) return;
    const int split = blockIdx.y;
    const int per = (k.pnw + k.nsh - 1) / k.nsh;
    const int pbeg = k.pb0 + split * per, pend = min(k.pb0 + k.pnw, pbeg + per);
    const int deg = k.g.sh_degree;
    const int K = (deg + 1) * (deg + 1);
    const GaussRec rec = k.recs[gi];
    const float mu[3] = {rec.a.x, rec.a.y, rec.a.z};
    float f[KM];
    load_feat<KM>(k.g, gi, f);
    float dF[KM], dMu[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KM; ++c) dF[c] = 0.f;
    for (int p = pbeg; p < pend; ++p) {
        const float drho = k.drho[(size_t)(p - k.pb0) * k.g.ng + gi];
        if (drho == 0.f) continue;
        const float q[3] = {k.geo.wall[3 * p] - mu[0], k.geo.wall[3 * p + 1] - mu[1], k.geo.wall[3 * p + 2] - mu[2]};
        float dir[3], nrm;
        view_dir<PRESET>(-q[0], -q[1], -q[2], dir[0], dir[1], dir[2], nrm);
        float Y[KM];
        sh_basis<PRESET>(deg, dir[0], dir[1], dir[2], Y);
#pragma unroll
        for (int c = 0; c < KM; ++c)
            if (c < K) dF[c] += drho * Y[c];
        float gx, gy, gz;
        sh_grad_dir<PRESET>(deg, dir[0], dir[1], dir[2], f, gx, gy, gz);
        float ox, oy, oz;
        view_dir_bwd<PRESET>(-q[0], -q[1], -q[2], nrm, drho * gx, drho * gy, drho * gz, ox, oy, oz);
        dMu[0] += ox; dMu[1] += oy; dMu[2] += oz;
    }
    float* dst = k.shpart + ((size_t)split * k.g.ng + gi) * kShPart;
    if (k.accum) {
#pragma unroll
        for (int c = 0; c < KM; ++c) dst[c] += dF[c];
        dst[KM] += dMu[0]; dst[KM + 1] += dMu[1]; dst[KM + 2] += dMu[2];
    } else {
#pragma unroll
        for (int c = 0; c < KM; ++c) dst[c] = dF[c];
        dst[KM] = dMu[0]; dst[KM + 1] = dMu[1]; dst[KM + 2] = dMu[2];
    }
}

// ------------------------------------------------------------------------------------------
// finish: reduce the splits and chain dA / dsigma to the raw parameters
// ------------------------------------------------------------------------------------------
template <int PRESET, int KM>
__global__ __launch_bounds__(kBlock) void finish_kernel(KArgs k, float* d_mu, float* d_scaling, float* d_rot,
                                                        float* d_opac, float* d_feat) {
    const int i = k.g_lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k.g_hi) return;
    float acc[13 + KM];
    for (int t = 0; t < 13 + KM; ++t) acc[t] = 0.f;
    {
        // the wall-point splits' partials summed in fp64 (fixed order): the rotational shape sums are small
        // differences of the splits' contributions
        double sum[kBwdSlots];
        for (int t = 0; t < kBwdSlots; ++t) sum[t] = 0.0;
        for (int s = 0; s < k.nsplit; ++s) {
            const float* src = k.partial + ((size_t)s * k.g.ng + i) * 32;
            for (int t = 0; t < kBwdSlots; ++t) sum[t] += (double)src[t];
        }
        for (int t = 0; t < kBwdSlots; ++t) acc[t] = (float)sum[t];
    }
    for (int s = 0; s < k.nsh; ++s) {   // view-direction chain (sh_kernel)
        const float* src = k.shpart + ((size_t)s * k.g.ng + i) * kShPart;
        for (int t = 0; t < KM; ++t) acc[13 + t] += src[t];
        for (int t = 0; t < 3; ++t) acc[9 + t] += src[KM + t];
    }
    chain_to_raw_shape<PRESET>(k.g, i, acc, acc + 3, d_scaling, d_rot);
    d_mu[3 * i] = acc[9]; d_mu[3 * i + 1] = acc[10]; d_mu[3 * i + 2] = acc[11];
    const float sg = 1.0f / (1.0f + expf(-k.g.opacity[i]));
    d_opac[i] = acc[12] * sg * (1.0f - sg);
    const int kf = k.g.k_feat;
    const int K = (k.g.sh_degree + 1) * (k.g.sh_degree + 1);
#pragma unroll
    for (int c = 0; c < KM; ++c)
        if (c < kf) d_feat[(size_t)i * kf + c] = c < K ? acc[13 + c] : 0.f;
}


// 3-sigma AABB: bbox_compute.cuh:23-71 (cuda) / gaussian_model.py:140-178 (torch; clamp 1e-8)
template <int PRESET>
__global__ __launch_bounds__(kBlock) void bbox_kernel(nlosgr_gaussians g, float sig, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.ng) return;
    gauss_bbox<PRESET>(g, i, sig, out + 6 * (size_t)i);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------

bool bwd_shared(const nlosgr_geometry* geo, const nlosgr_options* opt);

int validate(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt) {
    if (!g || !geo || !opt) return set_err(NLOSGR_E_INVALID, "null argument struct");
    if (g->ng < 0) return set_err(NLOSGR_E_INVALID, "ng must be >= 0");
    if (g->preset != NLOSGR_PRESET_TORCH && g->preset != NLOSGR_PRESET_CUDA)
        return set_err(NLOSGR_E_INVALID, "unknown preset");
    // SH degree 4 exists in the torch preset only (sh_utils.py:102-112; spherical_harmonics.cuh stops at 3)
    const int max_deg = g->preset == NLOSGR_PRESET_TORCH ? 4 : 3;
    if (g->sh_degree < 0 || g->sh_degree > max_deg)
        return set_err(NLOSGR_E_UNSUPPORTED, g->preset == NLOSGR_PRESET_TORCH ? "active_sh_degree must be in [0, 4]"
                                                                              : "active_sh_degree must be in [0, 3] (cuda preset)");
    const int max_k = g->preset == NLOSGR_PRESET_TORCH ? kMaxK4 : kMaxK;
    if (g->k_feat < (g->sh_degree + 1) * (g->sh_degree + 1) || g->k_feat > max_k)
        return set_err(NLOSGR_E_INVALID, g->preset == NLOSGR_PRESET_TORCH ? "k_feat must satisfy (sh_degree+1)^2 <= k_feat <= 25"
                                                                           : "k_feat must satisfy (sh_degree+1)^2 <= k_feat <= 16");
    if (opt->mode != NLOSGR_MODE_NOOCL && opt->mode != NLOSGR_MODE_NETF && opt->mode != NLOSGR_MODE_BININT &&
        opt->mode != NLOSGR_MODE_OCCL)
        return set_err(NLOSGR_E_INVALID, "unknown mode");
    if (geo->nwall < 0 || geo->nt < 1 || geo->np < 1 || geo->nr < 1)
        return set_err(NLOSGR_E_INVALID, "bad geometry sizes");
    if (geo->nr > 4096 || geo->nt > 1024 || geo->np > 1024)
        return set_err(NLOSGR_E_UNSUPPORTED, "nr <= 4096 and nt, np <= 1024");
    if (g->ng > 0 && (!g->mu || !g->scaling || !g->rotation || !g->opacity || !g->features))
        return set_err(NLOSGR_E_INVALID, "null Gaussian parameter pointer");
    if (geo->nwall > 0 && (!geo->wall || !geo->sin_theta || !geo->cos_theta || !geo->sin_phi ||
                           !geo->cos_phi || !geo->grid_lin || !geo->hscale || !geo->r || !geo->att))
        return set_err(NLOSGR_E_INVALID, "null geometry pointer");
    if (tiles_engine(opt)) return tiles_validate(g, geo, opt);
    const size_t lds_f = (size_t)FwdLayout(geo->nr, geo->nt, geo->np).total * 4;
    const size_t lds_b = (size_t)BwdLayout(geo->nr, geo->nt, geo->np, bwd_shared(geo, opt)).total * 4;
    if (lds_f > 160 * 1024 || lds_b > 160 * 1024) return set_err(NLOSGR_E_UNSUPPORTED, "problem exceeds LDS budget");
    return NLOSGR_OK;
}

// shared-row backward layout when per-wave rows would leave fewer than 4 workgroups per CU
// (long rows, e.g. C5's 2048 bins); NLOSGR_FLAG_BWD_SHARED / _PERWAVE force either layout (A/B timing)
bool bwd_shared(const nlosgr_geometry* geo, const nlosgr_options* opt) {
    if (opt->flags & NLOSGR_FLAG_BWD_SHARED) return true;
    if (opt->flags & NLOSGR_FLAG_BWD_PERWAVE) return false;
    return (size_t)BwdLayout(geo->nr, geo->nt, geo->np).total * 4 > 40 * 1024;
}

int bwd_nsplit(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, bool shared) {
    const int maxs = geo->nwall > 0 ? geo->nwall : 1;
    if (opt->nsplit > 0) return opt->nsplit < maxs ? opt->nsplit : maxs;
    const int gpb = shared ? kNB * kWaves : kNB;
    const int nblk = (g->ng + gpb - 1) / gpb;
    // aim for ~48k workgroups: with 4 resident per CU a 3k-workgroup grid left a long last round
    // (C3 backward: 2 splits 354 ms, 16 -> 309, 32 -> 305, 64 -> 302)
    int ns = (49152 + nblk - 1) / (nblk > 0 ? nblk : 1);
    if (ns > maxs) ns = maxs;
    // per-wave layout: wave w walks wall points pbeg + w, + 4, ...; a split of fewer than 4 wall
    // points leaves waves idle while the workgroup still holds its LDS (small walls, e.g. C1's
    // 32x32: 1024 splits of one wall point ran one busy wave per workgroup)
    if (!shared && ns > maxs / kWaves) ns = maxs / kWaves;
    if (ns < 1) ns = 1;
    return ns;
}

// partial-slab splits the workspace layout reserves: the larger of the two layouts, so the ray
// cache's offset does not depend on which layout a later backward picks (NLOSGR_BSHARED)
// The backward runs over batches of wall points so that its dL/drho buffer ([batch][ng], read by
// sh_kernel) is bounded: NLOSGR_DRHO_MB (default 1024) MiB, i.e. C3 6.5 GB -> 1 GiB, a C5 rank 16.4 GB
// -> 1 GiB.  Split counts are sized for one batch; batches after the first add into the partial slabs.
int drho_batch(const nlosgr_gaussians* g, const nlosgr_geometry* geo) {
    const long long budget = (long long)(batch_budgets().drho_mb * 1048576.0);
    const long long per = (long long)(g->ng > 0 ? g->ng : 1) * (long long)sizeof(float);
    long long b = budget / per;
    if (b < 1) b = 1;
    if (b > geo->nwall) b = geo->nwall;
    return (int)(b > 0 ? b : 1);
}
nlosgr_geometry batch_geo(const nlosgr_gaussians* g, const nlosgr_geometry* geo) {
    nlosgr_geometry b = *geo;
    b.nwall = drho_batch(g, geo);
    return b;
}

int bwd_nsplit_ws(const nlosgr_gaussians* g, const nlosgr_geometry* geo0, const nlosgr_options* opt) {
    const nlosgr_geometry gb = batch_geo(g, geo0);
    const nlosgr_geometry* geo = &gb;
    const int a = bwd_nsplit(g, geo, opt, false), b = bwd_nsplit(g, geo, opt, true);
    return a > b ? a : b;
}


template <int PRESET, int MODE, bool DENSE, bool RAYS, bool CACHE>
void launch_fwd(const KArgs& ka, size_t shm, hipStream_t s) {
    const dim3 grid(ka.geo.nwall, (ka.hpart || ka.hfx) ? ka.nfsplit : 1);
    if constexpr ((MODE == NLOSGR_MODE_NOOCL || MODE == NLOSGR_MODE_NETF || MODE == NLOSGR_MODE_BININT) && !DENSE &&
                  !RAYS && !CACHE) {
        if (ka.hfx) {   // run_fwd decided the fixed-point TAIL drain (fx_eligible)
            hipLaunchKernelGGL((fwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE, true, true>), grid, dim3(kBlock), shm, s, ka);
            // the bright Gaussians' launch (one split per wall point; its list is usually empty)
            hipLaunchKernelGGL((fx_bright_kernel<PRESET, MODE>), dim3(ka.geo.nwall, 1), dim3(kBlock), shm, s, ka);
            return;
        }
    }
    constexpr bool kCanTail = (MODE == NLOSGR_MODE_NOOCL || MODE == NLOSGR_MODE_NETF || MODE == NLOSGR_MODE_BININT) &&
                              !DENSE && !RAYS;
    // NLOSGR_FLAG_MASKED_FWD: masked forward drain at every cutoff (A/B and parity cross-check); netf takes
    // the TAIL drain where its backward does (c dT <= 1/64), so both see the same support
    const bool tail = kCanTail && ka.opt.cutoff >= kTailCutoff && (!ka.counts || NLOSGR_FCOUNT_ON) &&
                      !(ka.opt.flags & NLOSGR_FLAG_MASKED_FWD) &&
                      (MODE != NLOSGR_MODE_NETF || ka.opt.c_deltaT <= kSmallX);
    if constexpr (!RAYS && !CACHE) {
        if (ka.counts) {   // nlosgr_count_support
            if (tail) hipLaunchKernelGGL((count_kernel<PRESET, MODE, DENSE, kCanTail>), grid, dim3(kBlock), shm, s, ka);
            else hipLaunchKernelGGL((count_kernel<PRESET, MODE, DENSE, false>), grid, dim3(kBlock), shm, s, ka);
            return;
        }
    }
    if (tail) hipLaunchKernelGGL((fwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE, kCanTail>), grid, dim3(kBlock), shm, s, ka);
    else hipLaunchKernelGGL((fwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE>), grid, dim3(kBlock), shm, s, ka);
}
template <int PRESET, int MODE, bool DENSE, bool RAYS, bool CACHE>
void launch_bwd(const KArgs& ka, size_t shm, hipStream_t s) {
    const int gpb = ka.bshared ? kNB * kWaves : kNB;
    dim3 grid((ka.g_hi - ka.g_lo + gpb - 1) / gpb, ka.nsplit);
    constexpr bool kCanTail = (MODE == NLOSGR_MODE_NOOCL || MODE == NLOSGR_MODE_NETF) && !DENSE && !RAYS;
    // NLOSGR_FLAG_MASKED_BWD: masked backward drains (A/B, parity cross-check)
    const bool tail = kCanTail && ka.opt.cutoff >= kTailCutoff && !(ka.opt.flags & NLOSGR_FLAG_MASKED_BWD) &&
                      (MODE != NLOSGR_MODE_NETF || ka.opt.c_deltaT <= kSmallX);
    if (ka.bshared) {
        if (tail) hipLaunchKernelGGL((bwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE, true, kCanTail>), grid, dim3(kBlock), shm, s, ka);
        else hipLaunchKernelGGL((bwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE, true>), grid, dim3(kBlock), shm, s, ka);
    } else {
        if (tail) hipLaunchKernelGGL((bwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE, false, kCanTail>), grid, dim3(kBlock), shm, s, ka);
        else hipLaunchKernelGGL((bwd_kernel<PRESET, MODE, DENSE, RAYS, CACHE, false>), grid, dim3(kBlock), shm, s, ka);
    }
}

// the ray cache is used only by the culled, histogram-only variants (the training hot path)
template <int PRESET, int MODE>
void dispatch_fwd(const KArgs& ka, bool dense, bool rays, size_t shm, hipStream_t s) {
    if (dense) {
        if (rays) launch_fwd<PRESET, MODE, true, true, false>(ka, shm, s);
        else launch_fwd<PRESET, MODE, true, false, false>(ka, shm, s);
    } else {
        if (rays) launch_fwd<PRESET, MODE, false, true, false>(ka, shm, s);
        else if (ka.cmask && MODE != NLOSGR_MODE_BININT) launch_fwd<PRESET, MODE, false, false, MODE != NLOSGR_MODE_BININT>(ka, shm, s);
        else launch_fwd<PRESET, MODE, false, false, false>(ka, shm, s);
    }
}
template <int PRESET, int MODE>
void dispatch_bwd(const KArgs& ka, bool dense, bool rays, size_t shm, hipStream_t s) {
    if (dense) {
        if (rays) launch_bwd<PRESET, MODE, true, true, false>(ka, shm, s);
        else launch_bwd<PRESET, MODE, true, false, false>(ka, shm, s);
    } else {
        if (rays) launch_bwd<PRESET, MODE, false, true, false>(ka, shm, s);
        else if (ka.cmask) launch_bwd<PRESET, MODE, false, false, true>(ka, shm, s);
        else launch_bwd<PRESET, MODE, false, false, false>(ka, shm, s);
    }
}


// workspace layout: GaussRec[ng] | backward partials [nsplit][ng][32] | ray cache (opt->ray_cache):
// mask 2 x u64 [P][ng] | box u32 [P][ng]
size_t cache_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt) {
    return opt->ray_cache ? align_up((size_t)geo->nwall * g->ng * 24) : 0;
}
// sh_kernel wall-point splits (>= 8 x 256-lane blocks per split row keep the chip busy at large Ng)
int sh_nsplit(const nlosgr_gaussians* g, const nlosgr_geometry* geo) {
    int ns = geo->nwall / 256;
    const int nblk = (g->ng + kBlock - 1) / kBlock;
    if (ns * nblk > 4096) ns = 4096 / (nblk > 0 ? nblk : 1);
    if (ns > 64) ns = 64;
    return ns < 1 ? 1 : ns;
}
// forward Gaussian splits per wall point: aim for 131072 workgroups (a 16k-workgroup grid of
// one long workgroup per wall point leaves a ragged last round), at least 256 Gaussians per split
#ifndef NLOSGR_FWD_SPLITS_MAX
#define NLOSGR_FWD_SPLITS_MAX 8        // forward Gaussian splits per wall point, at most
#endif
#ifndef NLOSGR_FWD_WG_TARGET
#define NLOSGR_FWD_WG_TARGET 131072    // forward workgroups aimed at (wall points x splits)
#endif
int fwd_nsplit(const nlosgr_gaussians* g, const nlosgr_geometry* geo) {
    if (geo->nwall <= 0) return 1;
    int ns = (NLOSGR_FWD_WG_TARGET + geo->nwall - 1) / geo->nwall;
    const int byg = (g->ng + 255) / 256;
    if (ns > byg) ns = byg;
    if (ns > NLOSGR_FWD_SPLITS_MAX) ns = NLOSGR_FWD_SPLITS_MAX;
    return ns < 1 ? 1 : ns;
}
// forward partials: float [nfsplit][P][nr] (float drains) or, for the FX drain, u64 [P][nr]; then the FX
// tail (bound histogram and info words, kFxTailBytes), the per-Gaussian bounds and the bright list
size_t fx_tail_off(const nlosgr_gaussians* g, const nlosgr_geometry* geo) {
    const int ns = fwd_nsplit(g, geo);
    const size_t fl = ns > 1 ? (size_t)ns * geo->nwall * geo->nr * sizeof(float) : 0;
    const size_t fx = (size_t)geo->nwall * geo->nr * sizeof(unsigned long long);
    return align_up(fl > fx ? fl : fx);
}
size_t fpart_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo) {
    return fx_tail_off(g, geo) + kFxTailBytes + 2 * align_up((size_t)g->ng * sizeof(float));
}
// the fixed-point TAIL drain serves the culled no-occlusion histogram at cutoff >= kTailCutoff
// (NLOSGR_FLAG_FLOAT_DRAIN: the float claim drain instead, A/B)
bool fx_eligible(const nlosgr_options* opt, bool dense, bool rays, bool counts, bool hist, bool cache) {
    const bool mode_ok = opt->mode == NLOSGR_MODE_NOOCL || opt->mode == NLOSGR_MODE_BININT ||
                         (opt->mode == NLOSGR_MODE_NETF && opt->c_deltaT <= kSmallX);   // (the TAIL drains)
    return mode_ok && opt->cutoff >= kTailCutoff && !dense && !rays && !counts && hist && !cache &&
           !(opt->flags & (NLOSGR_FLAG_FLOAT_DRAIN | NLOSGR_FLAG_MASKED_FWD));
}
// after the ray cache: drho [P][ng] | sh partials [nsh][ng][kShPart] | 256-B diagnostics tail |
// forward split partial histograms [nfsplit][P][nr]
size_t sh_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo0) {
    const nlosgr_geometry gb = batch_geo(g, geo0);   // dL/drho for one wall-point batch
    return align_up((size_t)gb.nwall * g->ng * sizeof(float)) +
           align_up((size_t)sh_nsplit(g, &gb) * g->ng * kShPart * sizeof(float));
}
// the forward partials / FX area (after the backward buffers and the 256-B diagnostics tail)
char* fpart_ptr(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* workspace) {
    return (char*)workspace + align_up((size_t)g->ng * sizeof(GaussRec)) +
           align_up((size_t)bwd_nsplit_ws(g, geo, opt) * g->ng * 32 * sizeof(float)) + cache_bytes(g, geo, opt) +
           sh_bytes(g, geo) + 256;
}
void cache_ptrs(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* ws, int nsplit,
                KArgs& ka) {
    if (!opt->ray_cache || g->ng == 0 || geo->nwall == 0) return;
    char* base = (char*)ws + align_up((size_t)g->ng * sizeof(GaussRec)) + align_up((size_t)nsplit * g->ng * 32 * sizeof(float));
    ka.cmask = (ulonglong2*)base;
    ka.cbox = (unsigned*)(base + (size_t)geo->nwall * g->ng * 16);
    ka.crho = (float*)(base + (size_t)geo->nwall * g->ng * 20);
}

int run_fwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* workspace,
            float* hist_out, float* ray_out, unsigned long long* counts, hipStream_t s) {
    if (g->ng > 0 && !workspace) return set_err(NLOSGR_E_INVALID, "workspace is null");
    KArgs ka;
    memset(&ka, 0, sizeof(ka));
    ka.g = *g; ka.geo = *geo; ka.opt = *opt;
    ka.recs = (const GaussRec*)workspace;
    ka.hist_out = hist_out; ka.ray_out = ray_out;
    ka.counts = counts;
    if (!counts) cache_ptrs(g, geo, opt, workspace, bwd_nsplit_ws(g, geo, opt), ka);
    const int nfs = fwd_nsplit(g, geo);
    const bool dense = !(opt->cutoff > 0.f);
    const bool rays = ray_out != nullptr;
    char* fpart = g->ng > 0 ? fpart_ptr(g, geo, opt, workspace) : nullptr;
    const bool fx = g->ng > 0 && fx_eligible(opt, dense, rays, counts != nullptr, hist_out != nullptr, ka.cmask != nullptr);
    if (fx) {
        ka.hfx = (unsigned long long*)fpart;
        unsigned* bins = (unsigned*)(fpart + fx_tail_off(g, geo));
        ka.fx_info = (int*)(bins + kFxBins);
        float* bound = (float*)((char*)bins + kFxTailBytes);
        int* blist = (int*)((char*)bound + align_up((size_t)g->ng * sizeof(float)));
        ka.fx_bound = bound;
        ka.fx_blist = blist;
        ka.nfsplit = nfs;
        HIPCHK(hipMemsetAsync(ka.hfx, 0, (size_t)geo->nwall * geo->nr * sizeof(unsigned long long), s));
        HIPCHK(hipMemsetAsync(bins, 0, kFxBins * sizeof(unsigned) + 8 * sizeof(int), s));
        const int nb = (g->ng + kBlock - 1) / kBlock;
        const float ascale = opt->mode == NLOSGR_MODE_NETF ? opt->c_deltaT : 1.0f;
        if (g->preset == NLOSGR_PRESET_TORCH)
            hipLaunchKernelGGL(fx_bound_kernel<NLOSGR_PRESET_TORCH>, dim3(nb), dim3(kBlock), 0, s, *g, ascale, bins, bound);
        else
            hipLaunchKernelGGL(fx_bound_kernel<NLOSGR_PRESET_CUDA>, dim3(nb), dim3(kBlock), 0, s, *g, ascale, bins, bound);
        HIPCHK(hipGetLastError());
        // E <= E(max) + range: a bright term < 2^(kFxBits + range) units, and a bin receives at most
        // ceil(ng / 256) x nt x np bright terms per wall point, so its u64 sum stays below 2^63
        int range = kFxRange;
        {
            const double nterm = (double)((g->ng + 255) / 256) * (double)geo->nt * (double)geo->np;
            int bits = 0;
            while (bits < 63 && ldexp(1.0, bits) < nterm) ++bits;
            range = 63 - kFxBits - bits;
            range = range < 0 ? 0 : (range > kFxRange ? kFxRange : range);
        }
        hipLaunchKernelGGL(fx_unit_kernel, dim3(1), dim3(kFxBins), 0, s, bins, ka.fx_info,
                           (opt->flags & NLOSGR_FLAG_FX_MAXUNIT) ? 1 : 0, range);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(fx_blist_kernel, dim3(nb), dim3(kBlock), 0, s, bound, g->ng, ka.fx_info, blist);
        HIPCHK(hipGetLastError());
    } else if (hist_out && nfs > 1 && g->ng > 0) {
        ka.hpart = (float*)fpart;
        ka.nfsplit = nfs;
    }
    if (g->ng > 0) {
        // (FX: the bright Gaussians get a negative sigma in the records, see preprocess_kernel)
        launch_preprocess(g, (GaussRec*)workspace, s, ka.hfx ? ka.fx_bound : nullptr, ka.fx_info);
        HIPCHK(hipGetLastError());
    }
    const size_t shm = (size_t)FwdLayout(geo->nr, geo->nt, geo->np, fx).total * sizeof(float);
    // NLOSGR_FLAG_LANE_DENSE routes the dense histogram through fwd_kernel instead (parity cross-check)
    if (dense && !rays && !counts && hist_out && opt->mode == NLOSGR_MODE_NOOCL && geo->nr <= 1024 &&
        !(opt->flags & NLOSGR_FLAG_LANE_DENSE)) {
        // dense no-occlusion histogram: lane = bin register accumulation (fwd_dense_kernel)
        if (g->ng > 0 && geo->nwall > 0) {
            const size_t shd = (size_t)FwdDenseLayout(geo->nr, geo->nt, geo->np).total * sizeof(float);
            const dim3 grid(geo->nwall, ka.hpart ? ka.nfsplit : 1);
            const int nb = (geo->nr + 63) / 64;
            const bool tp = g->preset == NLOSGR_PRESET_TORCH;
#define NLOSGR_FD(NBV)                                                                                   \
    do {                                                                                                 \
        if (tp) hipLaunchKernelGGL((fwd_dense_kernel<0, NBV>), grid, dim3(kBlock), shd, s, ka);          \
        else hipLaunchKernelGGL((fwd_dense_kernel<1, NBV>), grid, dim3(kBlock), shd, s, ka);             \
    } while (0)
            if (nb <= 1) NLOSGR_FD(1);
            else if (nb <= 2) NLOSGR_FD(2);
            else if (nb <= 4) NLOSGR_FD(4);
            else if (nb <= 8) NLOSGR_FD(8);
            else NLOSGR_FD(16);
#undef NLOSGR_FD
            HIPCHK(hipGetLastError());
        } else if (geo->nwall > 0) {
            HIPCHK(hipMemsetAsync(hist_out, 0, (size_t)geo->nwall * geo->nr * sizeof(float), s));
        }
        if (ka.hpart && g->ng > 0 && geo->nwall > 0) {
            const long long n = (long long)geo->nwall * geo->nr;
            hipLaunchKernelGGL(hist_reduce_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                               ka.hpart, ka.nfsplit, (long long)geo->nwall, geo->nr, geo->att, geo->hscale, hist_out);
            HIPCHK(hipGetLastError());
        }
        return NLOSGR_OK;
    }
    if (g->preset == NLOSGR_PRESET_TORCH) {
        if (opt->mode == NLOSGR_MODE_NOOCL) dispatch_fwd<0, 0>(ka, dense, rays, shm, s);
        else if (opt->mode == NLOSGR_MODE_NETF) dispatch_fwd<0, 1>(ka, dense, rays, shm, s);
        else dispatch_fwd<0, 2>(ka, dense, rays, shm, s);
    } else {
        if (opt->mode == NLOSGR_MODE_NOOCL) dispatch_fwd<1, 0>(ka, dense, rays, shm, s);
        else if (opt->mode == NLOSGR_MODE_NETF) dispatch_fwd<1, 1>(ka, dense, rays, shm, s);
        else dispatch_fwd<1, 2>(ka, dense, rays, shm, s);
    }
    HIPCHK(hipGetLastError());
    if (ka.hfx) {
        const long long n = (long long)geo->nwall * geo->nr;
        hipLaunchKernelGGL(fx_reduce_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ka.hfx,
                           ka.fx_info, (long long)geo->nwall, geo->nr, geo->att, geo->hscale, hist_out);
        HIPCHK(hipGetLastError());
    } else if (ka.hpart) {
        const long long n = (long long)geo->nwall * geo->nr;
        hipLaunchKernelGGL(hist_reduce_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ka.hpart,
                           ka.nfsplit, (long long)geo->nwall, geo->nr, geo->att, geo->hscale, hist_out);
        HIPCHK(hipGetLastError());
    }
    return NLOSGR_OK;
}

}  // namespace

extern "C" {

int nlosgr_abi_version(void) { return NLOSGR_ABI_VERSION; }

#ifdef NLOSGR_FXCOUNT
__attribute__((visibility("default"))) int nlosgr_debug_fx_counts(unsigned long long* out8) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_fdbg), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fdbg), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef NLOSGR_BCOUNT
__attribute__((visibility("default"))) int nlosgr_debug_bwd_counts(unsigned long long* out8) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_bdbg), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_bdbg), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

void nlosgr_set_batch_budgets(double drho_mb, double tile_hpart_mb) {
    BatchBudgets& b = batch_budgets();
    if (drho_mb > 0.0) b.drho_mb = drho_mb;
    if (tile_hpart_mb > 0.0) b.tile_hpart_mb = tile_hpart_mb;
}

void nlosgr_get_batch_budgets(double* drho_mb, double* tile_hpart_mb) {
    const BatchBudgets& b = batch_budgets();
    if (drho_mb) *drho_mb = b.drho_mb;
    if (tile_hpart_mb) *tile_hpart_mb = b.tile_hpart_mb;
}

const char* nlosgr_last_error(void) { return g_err; }

size_t nlosgr_workspace_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt) {
    if (validate(g, geo, opt) != NLOSGR_OK) return 0;
    if (tiles_engine(opt)) return tiles_workspace_bytes(g, geo, opt);
    const size_t rec = align_up((size_t)g->ng * sizeof(GaussRec));
    const size_t part = align_up((size_t)bwd_nsplit_ws(g, geo, opt) * g->ng * 32 * sizeof(float));
    return rec + part + cache_bytes(g, geo, opt) + sh_bytes(g, geo) + 256 + fpart_bytes(g, geo);
}

int nlosgr_render_fwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt,
                      void* workspace, float* hist_out, float* ray_out, void* hip_stream) {
    const int rc = validate(g, geo, opt);
    if (rc) return rc;
    if (geo->nwall == 0 || (!hist_out && !ray_out)) return NLOSGR_OK;
    if (tiles_engine(opt)) return tiles_fwd(g, geo, opt, workspace, hist_out, ray_out, (hipStream_t)hip_stream);
    return run_fwd(g, geo, opt, workspace, hist_out, ray_out, nullptr, (hipStream_t)hip_stream);
}

int nlosgr_fx_info(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt,
                   const void* workspace, int32_t* info_out, void* hip_stream) {
    const int rc = validate(g, geo, opt);
    if (rc) return rc;
    if (!workspace || !info_out) return set_err(NLOSGR_E_INVALID, "null workspace or info_out");
    if (tiles_engine(opt) || g->ng == 0) return set_err(NLOSGR_E_UNSUPPORTED, "fx_info: pair-major forward with ng > 0");
    const char* fpart = fpart_ptr(g, geo, opt, const_cast<void*>(workspace));
    const char* info = fpart + fx_tail_off(g, geo) + kFxBins * sizeof(unsigned);
    HIPCHK(hipMemcpyAsync(info_out, info, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)hip_stream));
    return NLOSGR_OK;
}

int nlosgr_count_support(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt,
                         void* workspace, unsigned long long* counts, void* hip_stream) {
    const int rc = validate(g, geo, opt);
    if (rc) return rc;
    if (!counts) return set_err(NLOSGR_E_INVALID, "counts is null");
    if (tiles_engine(opt)) return set_err(NLOSGR_E_UNSUPPORTED, "count_support: pair-major modes only");
    hipStream_t s = (hipStream_t)hip_stream;
    HIPCHK(hipMemsetAsync(counts, 0, 3 * sizeof(unsigned long long), s));
    if (geo->nwall == 0) return NLOSGR_OK;
    return run_fwd(g, geo, opt, workspace, nullptr, nullptr, counts, s);
}

int nlosgr_render_bwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt,
                      void* workspace, const float* grad_hist, const float* grad_ray, float* d_mu,
                      float* d_scaling, float* d_rotation, float* d_opacity, float* d_features,
                      void* hip_stream) {
    int rc = validate(g, geo, opt);
    if (rc) return rc;
    if (opt->mode == NLOSGR_MODE_BININT)
        return set_err(NLOSGR_E_UNSUPPORTED, "no backward for the bin-integrated (analytic) forward");
    if (g->ng == 0) return NLOSGR_OK;
    if (!workspace) return set_err(NLOSGR_E_INVALID, "workspace is null");
    if (!d_mu || !d_scaling || !d_rotation || !d_opacity || !d_features)
        return set_err(NLOSGR_E_INVALID, "null gradient output pointer");
    if (opt->g_end > 0 && (opt->g_begin < 0 || opt->g_begin >= opt->g_end || opt->g_end > g->ng ||
                           opt->g_begin % 256 != 0 || tiles_engine(opt)))
        return set_err(NLOSGR_E_INVALID, "backward Gaussian range: 0 <= g_begin < g_end <= ng, g_begin % 256 == 0 "
                                         "(pair-major modes)");
    if (tiles_engine(opt))
        return tiles_bwd(g, geo, opt, workspace, grad_hist, grad_ray, d_mu, d_scaling, d_rotation, d_opacity,
                         d_features, (hipStream_t)hip_stream);
    hipStream_t s = (hipStream_t)hip_stream;
    KArgs ka;
    memset(&ka, 0, sizeof(ka));
    ka.g = *g; ka.geo = *geo; ka.opt = *opt;
    ka.recs = (const GaussRec*)workspace;
    ka.partial = (float*)((char*)workspace + align_up((size_t)g->ng * sizeof(GaussRec)));
    ka.grad_hist = grad_hist; ka.grad_ray = grad_ray;
    ka.g_lo = opt->g_end > 0 ? opt->g_begin : 0;
    ka.g_hi = opt->g_end > 0 ? opt->g_end : g->ng;
    ka.bshared = bwd_shared(geo, opt) ? 1 : 0;
    const nlosgr_geometry gbat = batch_geo(g, geo);
    ka.nsplit = bwd_nsplit(g, &gbat, opt, ka.bshared != 0);
    cache_ptrs(g, geo, opt, workspace, bwd_nsplit_ws(g, geo, opt), ka);
    {
        char* shb = (char*)workspace + align_up((size_t)g->ng * sizeof(GaussRec)) +
                    align_up((size_t)bwd_nsplit_ws(g, geo, opt) * g->ng * 32 * sizeof(float)) + cache_bytes(g, geo, opt);
        ka.drho = (float*)shb;
        ka.shpart = (float*)(shb + align_up((size_t)gbat.nwall * g->ng * sizeof(float)));   // drho: one batch
        ka.nsh = sh_nsplit(g, &gbat);
        if (opt->flags & 8) {   // diagnostics: counters in the workspace's 256-B tail
            ka.counts = (unsigned long long*)(shb + sh_bytes(g, geo));
            HIPCHK(hipMemsetAsync(ka.counts, 0, 8 * sizeof(unsigned long long), s));
        }
    }
    launch_preprocess(g, (GaussRec*)workspace, s);
    HIPCHK(hipGetLastError());
    if (geo->nwall > 0 && (grad_hist || grad_ray)) {
        const size_t shm = (size_t)BwdLayout(geo->nr, geo->nt, geo->np, ka.bshared != 0).total * sizeof(float);
        const bool dense = !(opt->cutoff > 0.f);
        const bool rays = grad_ray != nullptr;
        const dim3 shgrid((ka.g_hi - ka.g_lo + kBlock - 1) / kBlock, ka.nsh);
        for (int pb0 = 0; pb0 < geo->nwall; pb0 += gbat.nwall) {   // wall-point batches (drho_batch)
            ka.pb0 = pb0;
            ka.pnw = geo->nwall - pb0 < gbat.nwall ? geo->nwall - pb0 : gbat.nwall;
            ka.accum = pb0 > 0 ? 1 : 0;
            if (g->preset == NLOSGR_PRESET_TORCH) {
                if (opt->mode == NLOSGR_MODE_NOOCL) dispatch_bwd<0, 0>(ka, dense, rays, shm, s);
                else dispatch_bwd<0, 1>(ka, dense, rays, shm, s);
            } else {
                if (opt->mode == NLOSGR_MODE_NOOCL) dispatch_bwd<1, 0>(ka, dense, rays, shm, s);
                else dispatch_bwd<1, 1>(ka, dense, rays, shm, s);
            }
            HIPCHK(hipGetLastError());
            if (g->preset == NLOSGR_PRESET_TORCH && g->sh_degree == 4)
                hipLaunchKernelGGL((sh_kernel<NLOSGR_PRESET_TORCH, kMaxK4>), shgrid, dim3(kBlock), 0, s, ka);
            else if (g->preset == NLOSGR_PRESET_TORCH)
                hipLaunchKernelGGL((sh_kernel<NLOSGR_PRESET_TORCH, kMaxK>), shgrid, dim3(kBlock), 0, s, ka);
            else
                hipLaunchKernelGGL((sh_kernel<NLOSGR_PRESET_CUDA, kMaxK>), shgrid, dim3(kBlock), 0, s, ka);
            HIPCHK(hipGetLastError());
        }
    } else {
        HIPCHK(hipMemsetAsync(ka.partial, 0, (size_t)ka.nsplit * g->ng * 32 * sizeof(float), s));
        ka.nsh = 0;
    }
    const int nb = (ka.g_hi - ka.g_lo + kBlock - 1) / kBlock;
    if (g->preset == NLOSGR_PRESET_TORCH && g->sh_degree == 4)
        hipLaunchKernelGGL((finish_kernel<NLOSGR_PRESET_TORCH, kMaxK4>), dim3(nb), dim3(kBlock), 0, s, ka, d_mu,
                           d_scaling, d_rotation, d_opacity, d_features);
    else if (g->preset == NLOSGR_PRESET_TORCH)
        hipLaunchKernelGGL((finish_kernel<NLOSGR_PRESET_TORCH, kMaxK>), dim3(nb), dim3(kBlock), 0, s, ka, d_mu,
                           d_scaling, d_rotation, d_opacity, d_features);
    else
        hipLaunchKernelGGL((finish_kernel<NLOSGR_PRESET_CUDA, kMaxK>), dim3(nb), dim3(kBlock), 0, s, ka, d_mu,
                           d_scaling, d_rotation, d_opacity, d_features);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

int nlosgr_bboxes(const nlosgr_gaussians* g, float sigma_scale, float* bboxes_out, void* hip_stream) {
    if (!g || !bboxes_out) return set_err(NLOSGR_E_INVALID, "null argument");
    if (g->ng <= 0) return NLOSGR_OK;
    hipStream_t s = (hipStream_t)hip_stream;
    const int nb = (g->ng + kBlock - 1) / kBlock;
    if (g->preset == NLOSGR_PRESET_TORCH)
        hipLaunchKernelGGL(bbox_kernel<NLOSGR_PRESET_TORCH>, dim3(nb), dim3(kBlock), 0, s, *g, sigma_scale, bboxes_out);
    else
        hipLaunchKernelGGL(bbox_kernel<NLOSGR_PRESET_CUDA>, dim3(nb), dim3(kBlock), 0, s, *g, sigma_scale, bboxes_out);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

}  // extern "C"

// Helpers shared by the translation units of libnlosgr (volume kernels, rays kernels):
// error state of the C ABI, wave-level primitives, hardware fast math, the parameter
// preprocessing kernel and the chain from dL/dA, dL/dsigma to the raw parameters.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nlosgr_device.hpp"

namespace nlosgr {
namespace detail {

inline thread_local char g_err[512] = "";

inline int set_err(int code, const char* msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return code;
}

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kMaxK = 16;      // SH coefficients up to degree 3 (cuda preset, path C / A kernels)
constexpr int kNB = 64;          // Gaussians per backward workgroup
constexpr float kPi = 3.14159265358979323846f;
constexpr float kHalfLog2e = 0.72134752044448170368f;  // log2(e)/2

// float -> int index, saturated before the conversion (no UB for huge / non-finite values)
__device__ __forceinline__ int fidx(float x, int lo, int hi) {
    x = fminf(fmaxf(x, (float)lo), (float)hi);
    return (int)x;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int lanes_below(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0));
}

// orders LDS traffic between lanes of one wave (no workgroup barrier needed)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ------------------------------------------------------------------------------------------
// fast math (hardware v_rcp / v_sqrt / v_exp / v_log, ~1 ulp) and a polynomial atan2
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float flog2(float x) { return __builtin_amdgcn_logf(x); }

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Batch budgets that shape the workspace layout (MiB): the backward's dL/drho wall-point batches and
// the ray-tile forward's partial histograms.  Defaults 1024 MiB each; changes go through
// nlosgr_set_batch_budgets only (ABI 8: no environment variables, so the batch boundaries, and with
// them the gradients' summation order, never depend on the caller's environment), so a workspace sized
// by nlosgr_workspace_bytes and a ray-cache backward see the layout of the forward that filled it.
struct BatchBudgets {
    double drho_mb = 1024.0, tile_hpart_mb = 1024.0;
};
inline BatchBudgets& batch_budgets() {
    static BatchBudgets b;
    return b;
}

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) return set_err(NLOSGR_E_HIP, hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------------------------------
// preprocess: raw params -> A = diag(1/s~) R', sigma, s_max, N = A^T A
// ------------------------------------------------------------------------------------------
// fxb / fxinfo (the forward's fixed-point drain, nlosgr_volume.hip kFxBits): a Gaussian whose amplitude bound
// reaches 2^24 units (fxb[i] x 2^E x 1.002 >= 2^24, E = fxinfo[0]) is stored with a negative sigma, so the
// main fixed-point launch skips it (w = sigma rho <= 0) and the bright launch takes |sigma|
template <int PRESET>
__global__ __launch_bounds__(kBlock) void preprocess_kernel(nlosgr_gaussians g, GaussRec* recs, const float* fxb,
                                                           const int* fxinfo) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.ng) return;
    float S[3] = {g.scaling[3 * i], g.scaling[3 * i + 1], g.scaling[3 * i + 2]};
    float Q[4] = {g.rotation[4 * i], g.rotation[4 * i + 1], g.rotation[4 * i + 2], g.rotation[4 * i + 3]};
    GaussAct a;
    activate<PRESET>(S, Q, g.opacity[i], g.scaling_modifier, a);
    float A[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) A[3 * r + c] = a.Rp[3 * r + c] / a.st[r];
    float N[6];
    const int ix[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
    for (int t = 0; t < 6; ++t) {
        const int p = ix[t][0], q = ix[t][1];
        N[t] = A[p] * A[q] + A[3 + p] * A[3 + q] + A[6 + p] * A[6 + q];
    }
    const float smax = fmaxf(a.st[0], fmaxf(a.st[1], a.st[2]));
    GaussRec rec;
    float sg = a.sigma;
    if (fxb && !(fxb[i] * ldexpf(1.0f, fxinfo[0]) * 1.002f < 16777216.0f)) sg = -sg;
    rec.a = make_float4(g.mu[3 * i], g.mu[3 * i + 1], g.mu[3 * i + 2], sg);
    rec.b = make_float4(A[0], A[1], A[2], A[3]);
    rec.c = make_float4(A[4], A[5], A[6], A[7]);
    rec.d = make_float4(A[8], smax, N[0], N[1]);
    rec.e = make_float4(N[2], N[3], N[4], N[5]);
    recs[i] = rec;
}

inline void launch_preprocess(const nlosgr_gaussians* g, GaussRec* recs, hipStream_t s, const float* fxb = nullptr,
                              const int* fxinfo = nullptr) {
    const int nb = (g->ng + kBlock - 1) / kBlock;
    if (g->preset == NLOSGR_PRESET_TORCH)
        hipLaunchKernelGGL(preprocess_kernel<NLOSGR_PRESET_TORCH>, dim3(nb), dim3(kBlock), 0, s, *g, recs, fxb, fxinfo);
    else
        hipLaunchKernelGGL(preprocess_kernel<NLOSGR_PRESET_CUDA>, dim3(nb), dim3(kBlock), 0, s, *g, recs, fxb, fxinfo);
}

// sig-sigma axis-aligned box of Gaussian i: bbox_compute.cuh:23-71 (cuda: s = exp(S) mod, identity for a
// zero quaternion) / gaussian_model.py:140-178 (torch: F.normalize then build_rotation, clamp 1e-8).
// out = (min xyz, max xyz)
template <int PRESET>
__device__ __forceinline__ void gauss_bbox(const nlosgr_gaussians& g, int i, float sig, float* out) {
    float s[3];
    for (int t = 0; t < 3; ++t) s[t] = expf(g.scaling[3 * i + t]) * g.scaling_modifier;
    const float* Q = g.rotation + 4 * i;
    float n = sqrtf(Q[0] * Q[0] + Q[1] * Q[1] + Q[2] * Q[2] + Q[3] * Q[3]);
    float R[9];
    if (PRESET == NLOSGR_PRESET_CUDA && n < 1e-8f) {
        R[0] = 1.f; R[1] = 0.f; R[2] = 0.f; R[3] = 0.f; R[4] = 1.f; R[5] = 0.f; R[6] = 0.f; R[7] = 0.f; R[8] = 1.f;
    } else {
        if (PRESET == NLOSGR_PRESET_TORCH) n = fmaxf(n, 1e-12f);
        float q[4] = {Q[0] / n, Q[1] / n, Q[2] / n, Q[3] / n};
        if (PRESET == NLOSGR_PRESET_TORCH) {
            const float n1 = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            for (int t = 0; t < 4; ++t) q[t] /= n1;
        }
        quat_rot(q[0], q[1], q[2], q[3], R);
    }
    for (int r = 0; r < 3; ++r) {
        float v = 0.f;
        for (int c = 0; c < 3; ++c) v += (R[3 * r + c] * s[c]) * (R[3 * r + c] * s[c]);
        if (PRESET == NLOSGR_PRESET_TORCH) v = fmaxf(v, 1e-8f);
        const float e = sig * sqrtf(v);
        out[r] = g.mu[3 * i + r] - e;
        out[3 + r] = g.mu[3 * i + r] + e;
    }
}

// dL/dR' (dRp[9]) and dL/ds~ (dst[3]) -> dL/d_scaling, dL/d_rotation of Gaussian i under the preset
template <int PRESET>
__device__ void chain_core(const nlosgr_gaussians& g, int i, const GaussAct& a, const float* dRp, const float* dst,
                           float* d_scaling, float* d_rot) {
    const float* S = g.scaling + 3 * i;
    const float* Q = g.rotation + 4 * i;
    const float mod = g.scaling_modifier;
    float dR[9];
    if (PRESET == NLOSGR_PRESET_TORCH) {
        for (int t = 0; t < 9; ++t) dR[t] = dRp[t];
        for (int r = 0; r < 3; ++r) {
            const float e = expf(S[r]) * mod;     // s = exp(e), ds/dS = s * e
            d_scaling[3 * i + r] = dst[r] * a.st[r] * e;
        }
        // q^ = Q / max(|Q|,1e-12); qn = q^/|q^|; R = R(qn)
        const float n0 = sqrtf(Q[0] * Q[0] + Q[1] * Q[1] + Q[2] * Q[2] + Q[3] * Q[3]);
        const float d0 = fmaxf(n0, 1e-12f);
        float qh[4] = {Q[0] / d0, Q[1] / d0, Q[2] / d0, Q[3] / d0};
        const float n1 = sqrtf(qh[0] * qh[0] + qh[1] * qh[1] + qh[2] * qh[2] + qh[3] * qh[3]);
        float qn[4] = {qh[0] / n1, qh[1] / n1, qh[2] / n1, qh[3] / n1};
        float dqn[4];
        quat_rot_bwd(qn[0], qn[1], qn[2], qn[3], dR, dqn[0], dqn[1], dqn[2], dqn[3]);
        float dp = qn[0] * dqn[0] + qn[1] * dqn[1] + qn[2] * dqn[2] + qn[3] * dqn[3];
        float dqh[4];
        for (int t = 0; t < 4; ++t) dqh[t] = (dqn[t] - qn[t] * dp) / n1;
        if (n0 > 1e-12f) {
            float dp2 = qh[0] * dqh[0] + qh[1] * dqh[1] + qh[2] * dqh[2] + qh[3] * dqh[3];
            for (int t = 0; t < 4; ++t) d_rot[4 * i + t] = (dqh[t] - qh[t] * dp2) / n0;
        } else {
            for (int t = 0; t < 4; ++t) d_rot[4 * i + t] = dqh[t] / d0;
        }
    } else {
        // R' = R^T
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) dR[3 * c + r] = dRp[3 * r + c];
        for (int r = 0; r < 3; ++r) d_scaling[3 * i + r] = dst[r] * (a.st[r] - 1e-8f);  // s = exp(S) mod
        const float n = sqrtf(Q[0] * Q[0] + Q[1] * Q[1] + Q[2] * Q[2] + Q[3] * Q[3]);
        if (n < 1e-8f) {
            for (int t = 0; t < 4; ++t) d_rot[4 * i + t] = 0.f;
        } else {
            float qn[4] = {Q[0] / n, Q[1] / n, Q[2] / n, Q[3] / n};
            float dqn[4];
            quat_rot_bwd(qn[0], qn[1], qn[2], qn[3], dR, dqn[0], dqn[1], dqn[2], dqn[3]);
            float dp = qn[0] * dqn[0] + qn[1] * dqn[1] + qn[2] * dqn[2] + qn[3] * dqn[3];
            for (int t = 0; t < 4; ++t) d_rot[4 * i + t] = (dqn[t] - qn[t] * dp) / n;
        }
    }
}

// dL/dA (acc[0..8], A = diag(1/s~) R') -> dL/d_scaling, dL/d_rotation of Gaussian i under the preset
template <int PRESET>
__device__ void chain_to_raw(const nlosgr_gaussians& g, int i, const float* acc, float* d_scaling, float* d_rot) {
    GaussAct a;
    activate<PRESET>(g.scaling + 3 * i, g.rotation + 4 * i, g.opacity[i], g.scaling_modifier, a);
    // A_rc = R'_rc / s~_r
    float dRp[9], dst[3];
    for (int r = 0; r < 3; ++r) {
        float acc_s = 0.f;
        for (int c = 0; c < 3; ++c) {
            dRp[3 * r + c] = acc[3 * r + c] / a.st[r];
            acc_s += acc[3 * r + c] * a.Rp[3 * r + c];
        }
        dst[r] = -acc_s / (a.st[r] * a.st[r]);
    }
    chain_core<PRESET>(g, i, a, dRp, dst, d_scaling, d_rot);
}

// Scale ratios of A = diag(1/s~) R' from its row norms (|A_r| = 1/s~_r): r2 = s~2^2/s~1^2, r3 = s~3^2/s~1^2.
// No contraction, so the backward kernel and the finish compute the same ratios.
__device__ __forceinline__ void scale_ratios(const float* A, float& r2, float& r3) {
#pragma clang fp contract(off)
    const float n1 = A[0] * A[0] + A[1] * A[1] + A[2] * A[2];
    const float n2 = A[3] * A[3] + A[4] * A[4] + A[5] * A[5];
    const float n3 = A[6] * A[6] + A[7] * A[7] + A[8] * A[8];
    r2 = n1 * __builtin_amdgcn_rcpf(n2);   // (the same instruction sequence in every kernel that calls it)
    r3 = n1 * __builtin_amdgcn_rcpf(n3);
}

// The backward's shape accumulators (round 6).  A contribution to dL/dA is an outer product g b^T (g = dL/du0
// with b = p - mu, or g = dL/dv with b = the ray direction); in whitened form M = dA A^T = g w^T, w = A b.
// Only 6 of its 9 degrees of freedom reach the raw parameters: the diagonal D_r = g_r w_r (the scales:
// dL/ds~_r = -D_r / s~_r) and the antisymmetric part of Omega = dR' R'^T = S~^-1 M S~ (the rotation),
// accumulated per contribution as K~ = s~1^2 (Omega - Omega^T)_ij / (s~i s~j) ... scaled so only the ratios
// r = s~^2 / s~1^2 appear:  K~23 = r3 g2 w3 - r2 g3 w2,  K~31 = g3 w1 - r3 g1 w3,  K~12 = r2 g1 w2 - g2 w1.
// Summing dA itself (round 5) carried the large symmetric part into every add, so the small rotational part
// came out of a cancellation (TrainStep's ordered vs unordered backward differed by 3.6e-5 of max in
// d_rotation against 1.8e-7 elsewhere); the rotational sums here never hold the symmetric part.
__device__ __forceinline__ void shape_acc(const float* gv, const float* w, float r2, float r3, float* D, float* K) {
    D[0] = fmaf(gv[0], w[0], D[0]);
    D[1] = fmaf(gv[1], w[1], D[1]);
    D[2] = fmaf(gv[2], w[2], D[2]);
    K[0] += r3 * gv[1] * w[2] - r2 * gv[2] * w[1];
    K[1] += gv[2] * w[0] - r3 * gv[0] * w[2];
    K[2] += r2 * gv[0] * w[1] - gv[1] * w[0];
}

// (D[3], K~[3]) of shape_acc -> dL/d_scaling, dL/d_rotation: dL/ds~_r = -D_r / s~_r; dL/dR' = Omega_a R' with
// Omega_a = (Omega - Omega^T) / 2, (Omega - Omega^T)_ij = K~_ij / sqrt(r_i r_j) (its symmetric part never
// reaches the rotation: the quaternion's tangent space sees only the antisymmetric part of dR' R'^T)
template <int PRESET>
__device__ void chain_to_raw_shape(const nlosgr_gaussians& g, int i, const float* D, const float* K, float* d_scaling,
                                   float* d_rot) {
    GaussAct a;
    activate<PRESET>(g.scaling + 3 * i, g.rotation + 4 * i, g.opacity[i], g.scaling_modifier, a);
    float A[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) A[3 * r + c] = a.Rp[3 * r + c] / a.st[r];
    float r2, r3;
    scale_ratios(A, r2, r3);
    float dst[3];
    for (int r = 0; r < 3; ++r) dst[r] = -D[r] / a.st[r];
    const float w23 = 0.5f * K[0] / sqrtf(r2 * r3), w31 = 0.5f * K[1] / sqrtf(r3), w12 = 0.5f * K[2] / sqrtf(r2);
    const float Om[9] = {0.f, w12, -w31, -w12, 0.f, w23, w31, -w23, 0.f};
    float dRp[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            dRp[3 * r + c] = Om[3 * r] * a.Rp[c] + Om[3 * r + 1] * a.Rp[3 + c] + Om[3 * r + 2] * a.Rp[6 + c];
    chain_core<PRESET>(g, i, a, dRp, dst, d_scaling, d_rot);
}

// ray-tile engine (nlosgr_tiles.hip): NLOSGR_MODE_OCCL and NLOSGR_SELECT_AABB
bool tiles_engine(const nlosgr_options* opt);
int tiles_validate(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt);
size_t tiles_workspace_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt);
int tiles_fwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* ws,
              float* hist_out, float* ray_out, hipStream_t s);
int tiles_bwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt, void* ws,
              const float* grad_hist, const float* grad_ray, float* d_mu, float* d_scaling, float* d_rotation,
              float* d_opacity, float* d_features, hipStream_t s);

}  // namespace detail
}  // namespace nlosgr

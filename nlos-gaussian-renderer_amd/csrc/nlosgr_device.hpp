// Device helpers for the transient Gaussian NLOS renderer (gfx950 / CDNA4).
//
// Conventions: preset TORCH restates gaussian_model/gaussian_model.py,
// sh_utils.py and gaussian_utils.py; preset CUDA restates submodules/cuda_renderer/include/
// cuda_utils.cuh and spherical_harmonics.cuh.  Only the per-Gaussian preprocessing and the SH
// basis differ between presets; the per-sample inner loops are convention-free:
//     u(x) = A (x - mu),  pdf = exp(-|u|^2 / 2),  A = diag(1/s~) R'
// with R' = R (torch) or R^T (cuda) and s~ = s (torch) or s + 1e-8 (cuda).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nlosgr.h"

namespace nlosgr {

constexpr int kMaxK4 = 25;     // SH degree 4 (torch preset, sh_utils.py:102-112): batched volume path only
constexpr float kSH_C0 = 0.28209479177387814f;
constexpr float kSH_C1 = 0.4886025119029199f;
// 3DGS-signed constants (sh_utils.py:26-43)
constexpr float kC2_0 = 1.0925484305920792f, kC2_1 = -1.0925484305920792f, kC2_2 = 0.31539156525252005f,
                kC2_3 = -1.0925484305920792f, kC2_4 = 0.5462742152960396f;
constexpr float kC3_0 = -0.5900435899266435f, kC3_1 = 2.890611442640554f, kC3_2 = -0.4570457994644658f,
                kC3_3 = 0.3731763325901154f, kC3_4 = -0.4570457994644658f, kC3_5 = 1.445305721320277f,
                kC3_6 = -0.5900435899266435f;
// degree 4 (sh_utils.py:44-54; torch preset only)
constexpr float kC4_0 = 2.5033429417967046f, kC4_1 = -1.7701307697799304f, kC4_2 = 0.9461746957575601f,
                kC4_3 = -0.6690465435572892f, kC4_4 = 0.10578554691520431f, kC4_5 = -0.6690465435572892f,
                kC4_6 = 0.47308734787878004f, kC4_7 = -1.7701307697799304f, kC4_8 = 0.6258357354491761f;
// unsigned constants (spherical_harmonics.cuh:20-54)
constexpr float kU2_a = 1.0925484305920792f, kU2_b = 0.31539156525252005f, kU2_c = 0.5462742152960396f;
constexpr float kU3_a = 0.5900435899266435f, kU3_b = 2.890611442640554f, kU3_c = 0.4570457994644658f,
                kU3_d = 0.3731763325901154f, kU3_e = 1.445305721320277f;

// SH basis Y[0..K) for a direction, preset-specific polynomial forms.
// TORCH: sh_utils.py:74-100; CUDA: spherical_harmonics.cuh:20-54 (evaluated on the eps'd direction).
template <int PRESET>
__device__ __forceinline__ void sh_basis(int deg, float x, float y, float z, float* Y) {
    Y[0] = kSH_C0;
    if (deg < 1) return;
    if (PRESET == NLOSGR_PRESET_TORCH) {
        Y[1] = -kSH_C1 * y; Y[2] = kSH_C1 * z; Y[3] = -kSH_C1 * x;
    } else {
        Y[1] = kSH_C1 * y; Y[2] = kSH_C1 * z; Y[3] = kSH_C1 * x;
    }
    if (deg < 2) return;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    if (PRESET == NLOSGR_PRESET_TORCH) {
        Y[4] = kC2_0 * xy; Y[5] = kC2_1 * yz; Y[6] = kC2_2 * (2.0f * zz - xx - yy);
        Y[7] = kC2_3 * xz; Y[8] = kC2_4 * (xx - yy);
    } else {
        Y[4] = kU2_a * xy; Y[5] = kU2_a * yz; Y[6] = kU2_b * (3.0f * zz - 1.0f);
        Y[7] = kU2_a * xz; Y[8] = kU2_c * (xx - yy);
    }
    if (deg < 3) return;
    if (PRESET == NLOSGR_PRESET_TORCH) {
        Y[9] = kC3_0 * y * (3.0f * xx - yy);
        Y[10] = kC3_1 * xy * z;
        Y[11] = kC3_2 * y * (4.0f * zz - xx - yy);
        Y[12] = kC3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
        Y[13] = kC3_4 * x * (4.0f * zz - xx - yy);
        Y[14] = kC3_5 * z * (xx - yy);
        Y[15] = kC3_6 * x * (xx - 3.0f * yy);
    } else {
        Y[9] = kU3_a * y * (3.0f * xx - yy);
        Y[10] = kU3_b * xy * z;
        Y[11] = kU3_c * y * (5.0f * zz - 1.0f);
        Y[12] = kU3_d * z * (5.0f * zz - 3.0f);
        Y[13] = kU3_c * x * (5.0f * zz - 1.0f);
        Y[14] = kU3_e * z * (xx - yy);
        Y[15] = kU3_a * x * (xx - 3.0f * yy);
    }
    if (PRESET != NLOSGR_PRESET_TORCH || deg < 4) return;   // Y[16..24]: degree 4, torch preset only
    Y[16] = kC4_0 * xy * (xx - yy);
    Y[17] = kC4_1 * yz * (3.0f * xx - yy);
    Y[18] = kC4_2 * xy * (7.0f * zz - 1.0f);
    Y[19] = kC4_3 * yz * (7.0f * zz - 3.0f);
    Y[20] = kC4_4 * (zz * (35.0f * zz - 30.0f) + 3.0f);
    Y[21] = kC4_5 * xz * (7.0f * zz - 3.0f);
    Y[22] = kC4_6 * (xx - yy) * (7.0f * zz - 1.0f);
    Y[23] = kC4_7 * xz * (xx - 3.0f * yy);
    Y[24] = kC4_8 * (xx * (xx - 3.0f * yy) - yy * (3.0f * xx - yy));
}

// sum_c f[c] Y_c(x,y,z) for c < (deg+1)^2, accumulated in c order without a Y[] array: the degree
// tests are uniform branches and f (registers or a global row) is read only below (deg+1)^2.
template <int PRESET>
__device__ __forceinline__ float sh_dot(int deg, float x, float y, float z, const float* f) {
    float s = f[0] * kSH_C0;
    if (deg < 1) return s;
    const float sg = PRESET == NLOSGR_PRESET_TORCH ? -1.0f : 1.0f;
    s += f[1] * (sg * kSH_C1 * y);
    s += f[2] * (kSH_C1 * z);
    s += f[3] * (sg * kSH_C1 * x);
    if (deg < 2) return s;
    float Y[kMaxK4];
    sh_basis<PRESET>(deg < 3 ? 2 : deg, x, y, z, Y);
    s += f[4] * Y[4]; s += f[5] * Y[5]; s += f[6] * Y[6]; s += f[7] * Y[7]; s += f[8] * Y[8];
    if (deg < 3) return s;
#pragma unroll
    for (int c = 9; c < 16; ++c) s += f[c] * Y[c];
    if (PRESET != NLOSGR_PRESET_TORCH || deg < 4) return s;
#pragma unroll
    for (int c = 16; c < kMaxK4; ++c) s += f[c] * Y[c];
    return s;
}

// d/d(x,y,z) of sum_c f[c] Y_c(x,y,z) (same polynomial forms as sh_basis).
template <int PRESET>
__device__ __forceinline__ void sh_grad_dir(int deg, float x, float y, float z, const float* f,
                                            float& gx, float& gy, float& gz) {
    gx = gy = gz = 0.0f;
    if (deg < 1) return;
    if (PRESET == NLOSGR_PRESET_TORCH) {
        gy += -kSH_C1 * f[1]; gz += kSH_C1 * f[2]; gx += -kSH_C1 * f[3];
    } else {
        gy += kSH_C1 * f[1]; gz += kSH_C1 * f[2]; gx += kSH_C1 * f[3];
    }
    if (deg < 2) return;
    const float xx = x * x, yy = y * y, zz = z * z;
    if (PRESET == NLOSGR_PRESET_TORCH) {
        gx += kC2_0 * y * f[4]; gy += kC2_0 * x * f[4];
        gy += kC2_1 * z * f[5]; gz += kC2_1 * y * f[5];
        gx += -2.0f * kC2_2 * x * f[6]; gy += -2.0f * kC2_2 * y * f[6]; gz += 4.0f * kC2_2 * z * f[6];
        gx += kC2_3 * z * f[7]; gz += kC2_3 * x * f[7];
        gx += 2.0f * kC2_4 * x * f[8]; gy += -2.0f * kC2_4 * y * f[8];
    } else {
        gx += kU2_a * y * f[4]; gy += kU2_a * x * f[4];
        gy += kU2_a * z * f[5]; gz += kU2_a * y * f[5];
        gz += 6.0f * kU2_b * z * f[6];
        gx += kU2_a * z * f[7]; gz += kU2_a * x * f[7];
        gx += 2.0f * kU2_c * x * f[8]; gy += -2.0f * kU2_c * y * f[8];
    }
    if (deg < 3) return;
    if (PRESET == NLOSGR_PRESET_TORCH) {
        gx += kC3_0 * 6.0f * x * y * f[9];            gy += kC3_0 * (3.0f * xx - 3.0f * yy) * f[9];
        gx += kC3_1 * y * z * f[10];                  gy += kC3_1 * x * z * f[10];   gz += kC3_1 * x * y * f[10];
        gx += kC3_2 * (-2.0f * x * y) * f[11];        gy += kC3_2 * (4.0f * zz - xx - 3.0f * yy) * f[11];
        gz += kC3_2 * 8.0f * y * z * f[11];
        gx += kC3_3 * (-6.0f * x * z) * f[12];        gy += kC3_3 * (-6.0f * y * z) * f[12];
        gz += kC3_3 * (6.0f * zz - 3.0f * xx - 3.0f * yy) * f[12];
        gx += kC3_4 * (4.0f * zz - 3.0f * xx - yy) * f[13];
        gy += kC3_4 * (-2.0f * x * y) * f[13];        gz += kC3_4 * 8.0f * x * z * f[13];
        gx += kC3_5 * 2.0f * x * z * f[14];           gy += kC3_5 * (-2.0f * y * z) * f[14];
        gz += kC3_5 * (xx - yy) * f[14];
        gx += kC3_6 * (3.0f * xx - 3.0f * yy) * f[15]; gy += kC3_6 * (-6.0f * x * y) * f[15];
    } else {
        gx += kU3_a * 6.0f * x * y * f[9];            gy += kU3_a * (3.0f * xx - 3.0f * yy) * f[9];
        gx += kU3_b * y * z * f[10];                  gy += kU3_b * x * z * f[10];   gz += kU3_b * x * y * f[10];
        gy += kU3_c * (5.0f * zz - 1.0f) * f[11];     gz += kU3_c * 10.0f * y * z * f[11];
        gz += kU3_d * (15.0f * zz - 3.0f) * f[12];
        gx += kU3_c * (5.0f * zz - 1.0f) * f[13];     gz += kU3_c * 10.0f * x * z * f[13];
        gx += kU3_e * 2.0f * x * z * f[14];           gy += kU3_e * (-2.0f * y * z) * f[14];
        gz += kU3_e * (xx - yy) * f[14];
        gx += kU3_a * (3.0f * xx - 3.0f * yy) * f[15]; gy += kU3_a * (-6.0f * x * y) * f[15];
    }
    if (PRESET != NLOSGR_PRESET_TORCH || deg < 4) return;
    // degree 4: partial derivatives of the sh_utils.py:102-112 polynomials (x, y, z independent)
    const float xy = x * y, xz = x * z, yz = y * z;
    // C4_0 xy(xx - yy)
    gx += kC4_0 * y * (3.0f * xx - yy) * f[16];     gy += kC4_0 * x * (xx - 3.0f * yy) * f[16];
    // C4_1 yz(3xx - yy)
    gx += kC4_1 * 6.0f * xy * z * f[17];            gy += kC4_1 * z * (3.0f * xx - 3.0f * yy) * f[17];
    gz += kC4_1 * y * (3.0f * xx - yy) * f[17];
    // C4_2 xy(7zz - 1)
    gx += kC4_2 * y * (7.0f * zz - 1.0f) * f[18];   gy += kC4_2 * x * (7.0f * zz - 1.0f) * f[18];
    gz += kC4_2 * 14.0f * xy * z * f[18];
    // C4_3 yz(7zz - 3)
    gy += kC4_3 * z * (7.0f * zz - 3.0f) * f[19];   gz += kC4_3 * y * (21.0f * zz - 3.0f) * f[19];
    // C4_4 (zz(35zz - 30) + 3)
    gz += kC4_4 * z * (140.0f * zz - 60.0f) * f[20];
    // C4_5 xz(7zz - 3)
    gx += kC4_5 * z * (7.0f * zz - 3.0f) * f[21];   gz += kC4_5 * x * (21.0f * zz - 3.0f) * f[21];
    // C4_6 (xx - yy)(7zz - 1)
    gx += kC4_6 * 2.0f * x * (7.0f * zz - 1.0f) * f[22];  gy += kC4_6 * -2.0f * y * (7.0f * zz - 1.0f) * f[22];
    gz += kC4_6 * 14.0f * z * (xx - yy) * f[22];
    // C4_7 xz(xx - 3yy)
    gx += kC4_7 * z * (3.0f * xx - 3.0f * yy) * f[23];    gy += kC4_7 * -6.0f * xy * z * f[23];
    gz += kC4_7 * x * (xx - 3.0f * yy) * f[23];
    // C4_8 (xx(xx - 3yy) - yy(3xx - yy)) = x^4 - 6 x^2 y^2 + y^4
    gx += kC4_8 * (4.0f * xx * x - 12.0f * x * yy) * f[24];
    gy += kC4_8 * (4.0f * yy * y - 12.0f * xx * y) * f[24];
    (void)yz; (void)xz;
}

// Row-major R(q) for a unit quaternion (w,x,y,z): gaussian_utils.py:201-209 / cuda_utils.cuh:74-84.
__device__ __forceinline__ void quat_rot(float w, float x, float y, float z, float* R) {
    R[0] = 1.0f - 2.0f * (y * y + z * z); R[1] = 2.0f * (x * y - w * z); R[2] = 2.0f * (x * z + w * y);
    R[3] = 2.0f * (x * y + w * z); R[4] = 1.0f - 2.0f * (x * x + z * z); R[5] = 2.0f * (y * z - w * x);
    R[6] = 2.0f * (x * z - w * y); R[7] = 2.0f * (y * z + w * x); R[8] = 1.0f - 2.0f * (x * x + y * y);
}

// dL/dq for R = quat_rot(q) given dL/dR (row-major).
__device__ __forceinline__ void quat_rot_bwd(float w, float x, float y, float z, const float* dR,
                                             float& dw, float& dx, float& dy, float& dz) {
    dw = 2.0f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
    dx = 2.0f * (y * dR[1] + z * dR[2] + y * dR[3] - 2.0f * x * dR[4] - w * dR[5] + z * dR[6] + w * dR[7] -
                 2.0f * x * dR[8]);
    dy = 2.0f * (-2.0f * y * dR[0] + x * dR[1] + w * dR[2] + x * dR[3] + z * dR[5] - w * dR[6] + z * dR[7] -
                 2.0f * y * dR[8]);
    dz = 2.0f * (-2.0f * z * dR[0] - w * dR[1] + x * dR[2] + w * dR[3] - 2.0f * z * dR[4] + y * dR[5] +
                 x * dR[6] + y * dR[7]);
}

// Per-Gaussian activated state for a preset.  Writes s~ (divisor scales), R' (row-major, so
// u = diag(1/s~) R' (x - mu)), the normalised quaternion chain and sigma.
struct GaussAct {
    float st[3];   // s~
    float Rp[9];   // R'
    float sigma;
};

template <int PRESET>
__device__ __forceinline__ void activate(const float* S, const float* Q, float O, float mod, GaussAct& a) {
    if (PRESET == NLOSGR_PRESET_TORCH) {
        // gaussian_model.py:265-266,281: s = exp(exp(S)*mod); q^ = F.normalize(q); R = build_rotation(q^)
        for (int i = 0; i < 3; ++i) a.st[i] = expf(expf(S[i]) * mod);
        float n0 = sqrtf(Q[0] * Q[0] + Q[1] * Q[1] + Q[2] * Q[2] + Q[3] * Q[3]);
        float d0 = fmaxf(n0, 1e-12f);
        float qh[4] = {Q[0] / d0, Q[1] / d0, Q[2] / d0, Q[3] / d0};
        float n1 = sqrtf(qh[0] * qh[0] + qh[1] * qh[1] + qh[2] * qh[2] + qh[3] * qh[3]);
        quat_rot(qh[0] / n1, qh[1] / n1, qh[2] / n1, qh[3] / n1, a.Rp);
    } else {
        // cuda_utils.cuh:54-85,124-151 + volume_renderer.cu:150-154: s = exp(S)*mod, R^T, s+1e-8
        for (int i = 0; i < 3; ++i) a.st[i] = expf(S[i]) * mod + 1e-8f;
        float n = sqrtf(Q[0] * Q[0] + Q[1] * Q[1] + Q[2] * Q[2] + Q[3] * Q[3]);
        float R[9];
        if (n < 1e-8f) {
            R[0] = 1.f; R[1] = 0.f; R[2] = 0.f; R[3] = 0.f; R[4] = 1.f; R[5] = 0.f; R[6] = 0.f; R[7] = 0.f; R[8] = 1.f;
        } else {
            quat_rot(Q[0] / n, Q[1] / n, Q[2] / n, Q[3] / n, R);
        }
        a.Rp[0] = R[0]; a.Rp[1] = R[3]; a.Rp[2] = R[6];
        a.Rp[3] = R[1]; a.Rp[4] = R[4]; a.Rp[5] = R[7];
        a.Rp[6] = R[2]; a.Rp[7] = R[5]; a.Rp[8] = R[8];
    }
    a.sigma = 1.0f / (1.0f + expf(-O));
}

// Unit view direction mu - p and its norm; TORCH divides by the norm (gaussian_model.py:351-352),
// CUDA multiplies by 1/(norm+1e-8) (cuda_utils.cuh:48-51).
template <int PRESET>
__device__ __forceinline__ void view_dir(float dx, float dy, float dz, float& ox, float& oy, float& oz,
                                         float& nrm) {
    nrm = sqrtf(dx * dx + dy * dy + dz * dz);
    if (PRESET == NLOSGR_PRESET_TORCH) {
        ox = dx / nrm; oy = dy / nrm; oz = dz / nrm;
    } else {
        float inv = 1.0f / (nrm + 1e-8f);
        ox = dx * inv; oy = dy * inv; oz = dz * inv;
    }
}

// Backward of view_dir: dL/d(dvec) given dL/d(dir).
template <int PRESET>
__device__ __forceinline__ void view_dir_bwd(float dx, float dy, float dz, float nrm, float gx, float gy,
                                             float gz, float& ox, float& oy, float& oz) {
    if (PRESET == NLOSGR_PRESET_TORCH) {
        float inv = 1.0f / nrm;
        float ux = dx * inv, uy = dy * inv, uz = dz * inv;
        float dp = ux * gx + uy * gy + uz * gz;
        ox = (gx - ux * dp) * inv; oy = (gy - uy * dp) * inv; oz = (gz - uz * dp) * inv;
    } else {
        float den = nrm + 1e-8f;
        float inv = 1.0f / den;
        float dp = dx * gx + dy * gy + dz * gz;
        float c = (nrm > 0.0f) ? dp / (den * den * nrm) : 0.0f;
        ox = gx * inv - dx * c; oy = gy * inv - dy * c; oz = gz * inv - dz * c;
    }
}

// Packed per-Gaussian record written by the preprocess kernel (80 B).
struct __align__(16) GaussRec {
    float4 a;  // mu.xyz, sigma
    float4 b;  // A00 A01 A02 A10
    float4 c;  // A11 A12 A20 A21
    float4 d;  // A22, s_max (bounding-sphere scale), N00, N01   (N = A^T A = Sigma^-1)
    float4 e;  // N02, N11, N12, N22
};

}  // namespace nlosgr

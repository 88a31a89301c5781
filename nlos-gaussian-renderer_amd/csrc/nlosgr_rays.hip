// Path C "rays" API (gfx950): arbitrary rays x = o + t d through the Gaussians, per-(ray, sample)
// outputs — the semantics of the reference's _C.render_rays / filter_gaussians_per_ray
// (volume_renderer.cu:16-305, ray_aabb.cu:10-102, cuda_utils.cuh:97-151, bbox_compute.cuh:23-120)
// with a real backward (the reference's returns zeros, cuda_autograd.py:147-156).
//
//   filter : wave = one ray; lanes test 64 Gaussians' 3-sigma AABBs at a time (slab test of
//            cuda_utils.cuh:97-121) and append hits in index order, first 256 kept
//            (ray_aabb.cu:31-57).  Output layout [N_rays, 257]: count, indices, -1 padding.
//   forward: wave = one ray; the ray's Gaussians are staged in LDS as (u0 = A(o - mu), v = A d,
//            sigma, rho); lane = sample accumulates D = sum sigma pdf and the albedo-weighted
//            sum.  With occlusion the shared transmittance T_s = exp(-c dT sum_{s'<s} D_s') is an
//            exclusive wave scan; samples with T_s < 1e-4 are zero, as after the reference's
//            early exit (volume_renderer.cu:121-135).
//   backward: wave = one ray (one wave per workgroup: per-sample adjoints live in LDS); suffix
//            scan for dL/dD, then per Gaussian the sums over samples of dL/dpdf * pdf * z and
//            * t z, reduced across the wave.  Deterministic: a persistent grid of nslot
//            single-wave workgroups takes rays slot, slot + nslot, ... (static order) and adds
//            each (ray, Gaussian) result into the slot's private accumulator row (plain
//            read-modify-write, no atomics); a finish kernel sums the slot rows of each Gaussian
//            in slot order and chains them to the raw parameters (dA -> scaling/rotation,
//            dsigma -> opacity, drho -> SH / view direction).
#include "nlosgr_common.hpp"

using namespace nlosgr;
using namespace nlosgr::detail;

namespace {

constexpr int kMaxPerRay = NLOSGR_MAX_PER_RAY;
constexpr int kRowLen = kMaxPerRay + 1;
constexpr int kRayWaves = 4;           // forward / filter: rays per 256-thread workgroup
constexpr int kGD = 8;                 // floats per staged Gaussian: u0[3], v[3], sigma, rho

struct RArgs {
    nlosgr_gaussians g;
    nlosgr_rays r;
    const GaussRec* recs;
    const int32_t* filter;
    float cdt;
    float* acc;   // backward accumulators [nslot][ng][16]: dA[9], dMu[3], dsigma, drho
    int nslot;
};

// backward slots: at most 1024 single-wave workgroups and 1 GiB of accumulator rows
int rays_nslot(const nlosgr_gaussians* g, const nlosgr_rays* r) {
    const long long per = (long long)(g->ng > 0 ? g->ng : 1) * 16 * sizeof(float);
    long long n = (1ll << 30) / per;
    if (n > 1024) n = 1024;
    if (n > r->nrays) n = r->nrays;
    return n < 1 ? 1 : (int)n;
}

// ------------------------------------------------------------------------------------------
// AABB filter (first kMaxPerRay Gaussians by index whose box the half-infinite ray hits)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void filter_kernel(nlosgr_rays r, int ng, const float* __restrict__ bb,
                                                      int32_t* __restrict__ out) {
    const int ray = blockIdx.x * kRayWaves + (threadIdx.x >> 6);
    const int lane = lane_id();
    if (ray >= r.nrays) return;
    const float ox = r.origins[3 * ray], oy = r.origins[3 * ray + 1], oz = r.origins[3 * ray + 2];
    const float ix = 1.0f / (r.dirs[3 * ray] + 1e-8f);
    const float iy = 1.0f / (r.dirs[3 * ray + 1] + 1e-8f);
    const float iz = 1.0f / (r.dirs[3 * ray + 2] + 1e-8f);
    int32_t* row = out + (size_t)ray * kRowLen;
    int count = 0;
    for (int g0 = 0; g0 < ng && count < kMaxPerRay; g0 += 64) {
        const int g = g0 + lane;
        bool hit = false;
        if (g < ng) {
            const float* b = bb + 6 * (size_t)g;
            const float tx0 = (b[0] - ox) * ix, tx1 = (b[3] - ox) * ix;
            const float ty0 = (b[1] - oy) * iy, ty1 = (b[4] - oy) * iy;
            const float tz0 = (b[2] - oz) * iz, tz1 = (b[5] - oz) * iz;
            const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
            const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
            hit = tmax >= tmin && tmax >= 0.0f;
        }
        const unsigned long long m = __builtin_amdgcn_ballot_w64(hit);
        const int pos = count + lanes_below(m);
        if (hit && pos < kMaxPerRay) row[1 + pos] = g;
        count += __popcll(m);
    }
    if (count > kMaxPerRay) count = kMaxPerRay;
    for (int t = count + lane; t < kMaxPerRay; t += 64) row[1 + t] = -1;
    if (lane == 0) row[0] = count;
}

// ------------------------------------------------------------------------------------------
// per-(ray, Gaussian) staging: u0 = A (o - mu), v = A d, sigma, rho (SH albedo at mu - cam)
// ------------------------------------------------------------------------------------------
template <int PRESET>
__device__ __forceinline__ float albedo(const nlosgr_gaussians& g, int gi, float mx, float my, float mz,
                                        const float* cam, float& sh_out) {
    float dx, dy, dz, nrm;
    view_dir<PRESET>(mx - cam[0], my - cam[1], mz - cam[2], dx, dy, dz, nrm);
    float Y[kMaxK];
    sh_basis<PRESET>(g.sh_degree, dx, dy, dz, Y);
    const int K = (g.sh_degree + 1) * (g.sh_degree + 1);
    const float* f = g.features + (size_t)gi * g.k_feat;
    float sh = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxK; ++c)
        if (c < K) sh += f[c] * Y[c];
    sh_out = sh;
    return fmaxf(sh + 0.5f, 0.0f);
}

template <int PRESET>
__device__ __forceinline__ void stage_ray(const RArgs& k, int ray, const int32_t* list, int n, float* gd) {
    const float ox = k.r.origins[3 * ray], oy = k.r.origins[3 * ray + 1], oz = k.r.origins[3 * ray + 2];
    const float dx = k.r.dirs[3 * ray], dy = k.r.dirs[3 * ray + 1], dz = k.r.dirs[3 * ray + 2];
    for (int e = lane_id(); e < n; e += 64) {
        const int gi = list[e];
        const GaussRec rec = k.recs[gi];
        const float A[9] = {rec.b.x, rec.b.y, rec.b.z, rec.b.w, rec.c.x, rec.c.y, rec.c.z, rec.c.w, rec.d.x};
        const float q[3] = {ox - rec.a.x, oy - rec.a.y, oz - rec.a.z};
        float* o = gd + e * kGD;
        for (int r = 0; r < 3; ++r) {
            o[r] = A[3 * r] * q[0] + A[3 * r + 1] * q[1] + A[3 * r + 2] * q[2];
            o[3 + r] = A[3 * r] * dx + A[3 * r + 1] * dy + A[3 * r + 2] * dz;
        }
        float sh;
        o[6] = rec.a.w;
        o[7] = albedo<PRESET>(k.g, gi, rec.a.x, rec.a.y, rec.a.z, k.r.cam, sh);
    }
}

// D_s and the albedo-weighted sum W_s of one sample over the staged Gaussians
template <bool OCCL>
__device__ __forceinline__ void sample_sums(const float* gd, int n, float t, float cdt, float& D, float& W) {
    D = 0.f;
    W = 0.f;
    for (int e = 0; e < n; ++e) {
        const float4 a = *reinterpret_cast<const float4*>(gd + e * kGD);
        const float4 b = *reinterpret_cast<const float4*>(gd + e * kGD + 4);
        const float z0 = fmaf(t, a.w, a.x), z1 = fmaf(t, b.x, a.y), z2 = fmaf(t, b.y, a.z);
        const float m2 = fmaf(z0, z0, fmaf(z1, z1, z2 * z2));
        const float contrib = b.z * fast_exp2(-kHalfLog2e * m2);
        D += contrib;
        if (OCCL) W = fmaf(-expm1f(-contrib * cdt), b.w, W);
        else W = fmaf(contrib, b.w, W);
    }
}

template <int PRESET, bool OCCL>
__global__ __launch_bounds__(kBlock) void rays_fwd_kernel(RArgs k, float* __restrict__ rho_out,
                                                         float* __restrict__ dens_out, float* __restrict__ tr_out) {
    __shared__ __align__(16) float sm[kRayWaves * kMaxPerRay * kGD];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    const int ray = blockIdx.x * kRayWaves + wave;
    if (ray >= k.r.nrays) return;
    float* gd = sm + wave * kMaxPerRay * kGD;
    const int32_t* row = k.filter + (size_t)ray * kRowLen;
    const int n = min(max(row[0], 0), kMaxPerRay);
    stage_ray<PRESET>(k, ray, row + 1, n, gd);
    wave_sync();
    const int ns = k.r.nsamp;
    float carry = 0.f;   // c dT sum of D over earlier chunks
    for (int c0 = 0; c0 < ns; c0 += 64) {
        const int s = c0 + lane;
        const float t = s < ns ? k.r.t[s] : 0.f;
        float D, W;
        sample_sums<OCCL>(gd, n, t, k.cdt, D, W);
        if (s >= ns) D = W = 0.f;
        const size_t o = (size_t)ray * ns + s;
        if (!OCCL) {
            if (s < ns) {
                rho_out[o] = W * k.cdt;
                dens_out[o] = D;
                tr_out[o] = 1.0f;
            }
        } else {
            const float x = D * k.cdt;
            float incl = x;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const float u = __shfl_up(incl, off);
                if (lane >= off) incl += u;
            }
            const float T = expf(-(carry + incl - x));
            const bool live = T >= 1e-4f;
            if (s < ns) {
                rho_out[o] = live ? T * W : 0.f;
                dens_out[o] = live ? D : 0.f;
                tr_out[o] = live ? T : 0.f;
            }
            carry += __shfl(incl, 63);
        }
    }
}

// ------------------------------------------------------------------------------------------
// backward (one wave per workgroup)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <int PRESET, bool OCCL>
__global__ __launch_bounds__(64) void rays_bwd_kernel(RArgs k, const float* __restrict__ g_rho,
                                                     const float* __restrict__ g_dens,
                                                     const float* __restrict__ g_tr) {
    extern __shared__ __align__(16) float sm[];
    float* gd = sm;                               // [kMaxPerRay][kGD]
    float* GD = sm + kMaxPerRay * kGD;            // [ns] dL/dD_s
    float* GW = GD + k.r.nsamp;                   // [ns] dL/dW_s (W = the albedo-weighted sum)
    float* LV = GW + k.r.nsamp;                   // [ns] 1 where the sample is live (occlusion)
    const int lane = lane_id();
    float* acc_slot = k.acc + (size_t)blockIdx.x * k.g.ng * 16;
    for (int ray = blockIdx.x; ray < k.r.nrays; ray += k.nslot) {
        const int32_t* row = k.filter + (size_t)ray * kRowLen;
        const int n = min(max(row[0], 0), kMaxPerRay);
        if (n == 0) continue;
        wave_sync();   // the previous ray is done with the LDS tables
        stage_ray<PRESET>(k, ray, row + 1, n, gd);
        wave_sync();
        const int ns = k.r.nsamp;
        const float cdt = k.cdt;
        const size_t rbase = (size_t)ray * ns;
        if (!OCCL) {
            for (int s = lane; s < ns; s += 64) {
                GD[s] = g_dens ? g_dens[rbase + s] : 0.f;
                GW[s] = g_rho ? g_rho[rbase + s] * cdt : 0.f;
            }
        } else {
            // forward quantities, then dL/dD_s = g_D[s] - c dT sum_{s'>s} (g_rho rho + g_T T)_{s'}
            // over live samples (T_s >= 1e-4; the others are constant 0), dL/dW_s = g_rho[s] T_s
            float carry = 0.f;
            for (int c0 = 0; c0 < ns; c0 += 64) {
                const int s = c0 + lane;
                const float t = s < ns ? k.r.t[s] : 0.f;
                float D, W;
                sample_sums<true>(gd, n, t, cdt, D, W);
                if (s >= ns) D = W = 0.f;
                const float x = D * cdt;
                float incl = x;
    #pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const float u = __shfl_up(incl, off);
                    if (lane >= off) incl += u;
                }
                const float T = expf(-(carry + incl - x));
                const bool live = s < ns && T >= 1e-4f;
                const float gr = live && g_rho ? g_rho[rbase + s] : 0.f;
                const float gt = live && g_tr ? g_tr[rbase + s] : 0.f;
                if (s < ns) {
                    GW[s] = gr * T;
                    GD[s] = gr * T * W + gt * T;           // E_s, suffix-scanned below
                    LV[s] = live ? 1.f : 0.f;
                }
                carry += __shfl(incl, 63);
            }
            wave_sync();
            float suffix = 0.f;   // sum of E over later chunks
            for (int ch = (ns + 63) / 64 - 1; ch >= 0; --ch) {
                const int s = ch * 64 + lane;
                const float E = s < ns ? GD[s] : 0.f;
                float incl = E;   // inclusive suffix sum within the chunk
    #pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const float u = __shfl_down(incl, off);
                    if (lane + off < 64) incl += u;
                }
                if (s < ns) {
                    const float gdn = g_dens ? g_dens[rbase + s] : 0.f;
                    GD[s] = LV[s] != 0.f ? gdn - cdt * (suffix + incl - E) : 0.f;
                }
                suffix += __shfl(incl, 0);
            }
        }
        wave_sync();
        const float ox = k.r.origins[3 * ray], oy = k.r.origins[3 * ray + 1], oz = k.r.origins[3 * ray + 2];
        const float dxr = k.r.dirs[3 * ray], dyr = k.r.dirs[3 * ray + 1], dzr = k.r.dirs[3 * ray + 2];
        for (int e = 0; e < n; ++e) {
            const float4 a = *reinterpret_cast<const float4*>(gd + e * kGD);
            const float4 b = *reinterpret_cast<const float4*>(gd + e * kGD + 4);
            const float sig = b.z, rho = b.w;
            float Sz0 = 0.f, Sz1 = 0.f, Sz2 = 0.f, St0 = 0.f, St1 = 0.f, St2 = 0.f, dsig = 0.f, drho = 0.f;
            for (int s = lane; s < ns; s += 64) {
                const float t = k.r.t[s];
                const float z0 = fmaf(t, a.w, a.x), z1 = fmaf(t, b.x, a.y), z2 = fmaf(t, b.y, a.z);
                const float m2 = fmaf(z0, z0, fmaf(z1, z1, z2 * z2));
                const float pdf = fast_exp2(-kHalfLog2e * m2);
                const float contrib = sig * pdf;
                const float gD = GD[s], gW = GW[s];
                float dW_dc, wterm;   // dW/dcontrib and W's per-Gaussian term / rho
                if (OCCL) {
                    const float em = expf(-contrib * cdt);
                    dW_dc = rho * cdt * em;
                    wterm = -expm1f(-contrib * cdt);
                } else {
                    dW_dc = rho;
                    wterm = contrib;
                }
                const float gc = gD + gW * dW_dc;       // dL/dcontrib
                const float G = gc * sig * pdf;          // dL/dpdf * pdf
                Sz0 = fmaf(G, z0, Sz0); Sz1 = fmaf(G, z1, Sz1); Sz2 = fmaf(G, z2, Sz2);
                St0 = fmaf(G * t, z0, St0); St1 = fmaf(G * t, z1, St1); St2 = fmaf(G * t, z2, St2);
                dsig = fmaf(gc, pdf, dsig);
                drho = fmaf(gW, wterm, drho);
            }
            Sz0 = wave_sum(Sz0); Sz1 = wave_sum(Sz1); Sz2 = wave_sum(Sz2);
            St0 = wave_sum(St0); St1 = wave_sum(St1); St2 = wave_sum(St2);
            dsig = wave_sum(dsig); drho = wave_sum(drho);
            if (lane == 0) {
                // pdf = exp(-|z|^2/2), z = u0 + t v:  dL/du0 = -sum G z,  dL/dv = -sum G t z
                const int gi = row[1 + e];
                const GaussRec rec = k.recs[gi];
                const float A[9] = {rec.b.x, rec.b.y, rec.b.z, rec.b.w, rec.c.x, rec.c.y, rec.c.z, rec.c.w, rec.d.x};
                const float q[3] = {ox - rec.a.x, oy - rec.a.y, oz - rec.a.z};
                const float d3[3] = {dxr, dyr, dzr};
                const float dU[3] = {-Sz0, -Sz1, -Sz2}, dV[3] = {-St0, -St1, -St2};
                float* acc = acc_slot + (size_t)gi * 16;
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) acc[3 * r + c] += dV[r] * d3[c] + dU[r] * q[c];
                for (int c = 0; c < 3; ++c) acc[9 + c] += -(A[c] * dU[0] + A[3 + c] * dU[1] + A[6 + c] * dU[2]);
                acc[12] += dsig;
                acc[13] += drho;
            }
        }
    }
}

template <int PRESET>
__global__ __launch_bounds__(kBlock) void rays_finish_kernel(RArgs k, float* d_mu, float* d_scaling, float* d_rot,
                                                            float* d_opac, float* d_feat) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k.g.ng) return;
    float acc[16];
    for (int t = 0; t < 16; ++t) acc[t] = 0.f;
    for (int s = 0; s < k.nslot; ++s)
        for (int t = 0; t < 16; ++t) acc[t] += k.acc[((size_t)s * k.g.ng + i) * 16 + t];
    const float mx = k.g.mu[3 * i], my = k.g.mu[3 * i + 1], mz = k.g.mu[3 * i + 2];
    float dmu[3] = {acc[9], acc[10], acc[11]};
    const float drho = acc[13];
    // rho = max(0, 0.5 + SH(dir(mu - cam))); clamp_min passes the gradient where 0.5 + SH >= 0
    float dx, dy, dz, nrm;
    view_dir<PRESET>(mx - k.r.cam[0], my - k.r.cam[1], mz - k.r.cam[2], dx, dy, dz, nrm);
    float sh;
    albedo<PRESET>(k.g, i, mx, my, mz, k.r.cam, sh);
    const float gr = sh + 0.5f >= 0.f ? drho : 0.f;
    float Y[kMaxK];
    sh_basis<PRESET>(k.g.sh_degree, dx, dy, dz, Y);
    const int K = (k.g.sh_degree + 1) * (k.g.sh_degree + 1);
    const int kf = k.g.k_feat;
    for (int c = 0; c < kf; ++c) d_feat[(size_t)i * kf + c] = c < K ? gr * Y[c] : 0.f;
    if (gr != 0.f) {
        float gx, gy, gz;
        sh_grad_dir<PRESET>(k.g.sh_degree, dx, dy, dz, k.g.features + (size_t)i * kf, gx, gy, gz);
        float ox, oy, oz;
        view_dir_bwd<PRESET>(mx - k.r.cam[0], my - k.r.cam[1], mz - k.r.cam[2], nrm, gr * gx, gr * gy, gr * gz, ox,
                             oy, oz);
        dmu[0] += ox; dmu[1] += oy; dmu[2] += oz;
    }
    d_mu[3 * i] = dmu[0]; d_mu[3 * i + 1] = dmu[1]; d_mu[3 * i + 2] = dmu[2];
    const float sg = 1.0f / (1.0f + expf(-k.g.opacity[i]));
    d_opac[i] = acc[12] * sg * (1.0f - sg);
    chain_to_raw<PRESET>(k.g, i, acc, d_scaling, d_rot);
}

int validate_rays(const nlosgr_gaussians* g, const nlosgr_rays* r) {
    if (!g || !r) return set_err(NLOSGR_E_INVALID, "null argument struct");
    if (g->ng < 0 || r->nrays < 0 || r->nsamp < 0) return set_err(NLOSGR_E_INVALID, "negative size");
    if (g->preset != NLOSGR_PRESET_TORCH && g->preset != NLOSGR_PRESET_CUDA)
        return set_err(NLOSGR_E_INVALID, "unknown preset");
    if (g->sh_degree < 0 || g->sh_degree > 3)
        return set_err(NLOSGR_E_UNSUPPORTED, "active_sh_degree must be in [0, 3]");
    if (g->k_feat < (g->sh_degree + 1) * (g->sh_degree + 1) || g->k_feat > kMaxK)
        return set_err(NLOSGR_E_INVALID, "k_feat must satisfy (sh_degree+1)^2 <= k_feat <= 16");
    if (r->nsamp > 8192) return set_err(NLOSGR_E_UNSUPPORTED, "nsamp <= 8192");
    if (r->nrays > 0 && (!r->origins || !r->dirs || (r->nsamp > 0 && !r->t) || !r->cam))
        return set_err(NLOSGR_E_INVALID, "null ray pointer");
    if (g->ng > 0 && (!g->mu || !g->scaling || !g->rotation || !g->opacity || !g->features))
        return set_err(NLOSGR_E_INVALID, "null Gaussian parameter pointer");
    return NLOSGR_OK;
}

}  // namespace

extern "C" {

size_t nlosgr_rays_workspace_bytes(const nlosgr_gaussians* g, const nlosgr_rays* r) {
    if (validate_rays(g, r) != NLOSGR_OK) return 0;
    return align_up((size_t)g->ng * sizeof(GaussRec)) +
           align_up((size_t)rays_nslot(g, r) * g->ng * 16 * sizeof(float)) + 256;
}

int nlosgr_filter_rays(const nlosgr_gaussians* g, const nlosgr_rays* r, const float* bboxes, int32_t* filter_out,
                       void* hip_stream) {
    int rc = validate_rays(g, r);
    if (rc) return rc;
    if (r->nrays == 0) return NLOSGR_OK;
    if (!filter_out || (g->ng > 0 && !bboxes)) return set_err(NLOSGR_E_INVALID, "null filter/bbox pointer");
    hipStream_t s = (hipStream_t)hip_stream;
    hipLaunchKernelGGL(filter_kernel, dim3((r->nrays + kRayWaves - 1) / kRayWaves), dim3(kBlock), 0, s, *r, g->ng,
                       bboxes, filter_out);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

int nlosgr_rays_fwd(const nlosgr_gaussians* g, const nlosgr_rays* r, const int32_t* filter, float c_deltaT,
                    int32_t use_occlusion, void* workspace, float* rho_out, float* density_out, float* trans_out,
                    void* hip_stream) {
    int rc = validate_rays(g, r);
    if (rc) return rc;
    if (r->nrays == 0 || r->nsamp == 0) return NLOSGR_OK;
    if (!filter || !rho_out || !density_out || !trans_out) return set_err(NLOSGR_E_INVALID, "null output pointer");
    if (g->ng > 0 && !workspace) return set_err(NLOSGR_E_INVALID, "workspace is null");
    hipStream_t s = (hipStream_t)hip_stream;
    RArgs k;
    memset(&k, 0, sizeof(k));
    k.g = *g; k.r = *r; k.recs = (const GaussRec*)workspace; k.filter = filter; k.cdt = c_deltaT;
    if (g->ng > 0) launch_preprocess(g, (GaussRec*)workspace, s);
    const dim3 grid((r->nrays + kRayWaves - 1) / kRayWaves);
    if (g->preset == NLOSGR_PRESET_TORCH) {
        if (use_occlusion) hipLaunchKernelGGL((rays_fwd_kernel<0, true>), grid, dim3(kBlock), 0, s, k, rho_out, density_out, trans_out);
        else hipLaunchKernelGGL((rays_fwd_kernel<0, false>), grid, dim3(kBlock), 0, s, k, rho_out, density_out, trans_out);
    } else {
        if (use_occlusion) hipLaunchKernelGGL((rays_fwd_kernel<1, true>), grid, dim3(kBlock), 0, s, k, rho_out, density_out, trans_out);
        else hipLaunchKernelGGL((rays_fwd_kernel<1, false>), grid, dim3(kBlock), 0, s, k, rho_out, density_out, trans_out);
    }
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

int nlosgr_rays_bwd(const nlosgr_gaussians* g, const nlosgr_rays* r, const int32_t* filter, float c_deltaT,
                    int32_t use_occlusion, void* workspace, const float* g_rho, const float* g_density,
                    const float* g_trans, float* d_mu, float* d_scaling, float* d_rotation, float* d_opacity,
                    float* d_features, void* hip_stream) {
    int rc = validate_rays(g, r);
    if (rc) return rc;
    if (g->ng == 0) return NLOSGR_OK;
    if (!workspace || !filter) return set_err(NLOSGR_E_INVALID, "workspace/filter is null");
    if (!d_mu || !d_scaling || !d_rotation || !d_opacity || !d_features)
        return set_err(NLOSGR_E_INVALID, "null gradient output pointer");
    const size_t shm = (size_t)(kMaxPerRay * kGD + 3 * r->nsamp) * sizeof(float);
    if (shm > 160 * 1024) return set_err(NLOSGR_E_UNSUPPORTED, "nsamp exceeds the LDS budget");
    hipStream_t s = (hipStream_t)hip_stream;
    RArgs k;
    memset(&k, 0, sizeof(k));
    k.g = *g; k.r = *r; k.recs = (const GaussRec*)workspace; k.filter = filter; k.cdt = c_deltaT;
    k.acc = (float*)((char*)workspace + align_up((size_t)g->ng * sizeof(GaussRec)));
    k.nslot = rays_nslot(g, r);
    launch_preprocess(g, (GaussRec*)workspace, s);
    HIPCHK(hipMemsetAsync(k.acc, 0, (size_t)k.nslot * g->ng * 16 * sizeof(float), s));
    if (r->nrays > 0 && r->nsamp > 0 && (g_rho || g_density || g_trans)) {
        const dim3 grid(k.nslot);
        if (g->preset == NLOSGR_PRESET_TORCH) {
            if (use_occlusion) hipLaunchKernelGGL((rays_bwd_kernel<0, true>), grid, dim3(64), shm, s, k, g_rho, g_density, g_trans);
            else hipLaunchKernelGGL((rays_bwd_kernel<0, false>), grid, dim3(64), shm, s, k, g_rho, g_density, g_trans);
        } else {
            if (use_occlusion) hipLaunchKernelGGL((rays_bwd_kernel<1, true>), grid, dim3(64), shm, s, k, g_rho, g_density, g_trans);
            else hipLaunchKernelGGL((rays_bwd_kernel<1, false>), grid, dim3(64), shm, s, k, g_rho, g_density, g_trans);
        }
        HIPCHK(hipGetLastError());
    }
    const int nb = (g->ng + kBlock - 1) / kBlock;
    if (g->preset == NLOSGR_PRESET_TORCH)
        hipLaunchKernelGGL(rays_finish_kernel<0>, dim3(nb), dim3(kBlock), 0, s, k, d_mu, d_scaling, d_rotation, d_opacity, d_features);
    else
        hipLaunchKernelGGL(rays_finish_kernel<1>, dim3(nb), dim3(kBlock), 0, s, k, d_mu, d_scaling, d_rotation, d_opacity, d_features);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

}  // extern "C"

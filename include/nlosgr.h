/*
 * nlosgr.h — C ABI of the MI355X-native transient Gaussian NLOS renderer.
 *
 * Plain pointers and sizes only (no torch types).  Every device pointer is a gfx950 HBM
 * address owned by the caller; the library never allocates device memory: callers size the
 * scratch with nlosgr_workspace_bytes() and pass it in.  All work is enqueued on the given
 * HIP stream; no call synchronises the device.  Return value 0 = success, otherwise a
 * NLOSGR_E_* code with a message in nlosgr_last_error() (thread-local).
 *
 * Reference interfaces these entry points replace (paths under the reference repo):
 *   nlosgr_render_fwd   <- _C.render_rays            submodules/cuda_renderer/include/volume_renderer.h:8-24,
 *                                                    src/volume_renderer.cu:189-305
 *                       <- GaussianModel.estimate_rho_w_no_occlusion / estimate_rho_w('netf')
 *                          + gaussian_transient_rendering (the dense torch path that actually runs):
 *                          gaussian_model/gaussian_model.py:297-364, nlos_helpers.py:192-232
 *   nlosgr_render_bwd   <- CUDARenderFunction.backward gaussian_model/cuda_autograd.py:110-191
 *                          (zeros in the reference; real gradients here) and torch autograd of path T
 *   nlosgr_rays_analytic <- _C.render_rays_analytic  src/volume_renderer_analytic.cu:178-241
 *   nlosgr_mse / nlosgr_adam <- compute_loss nlos_helpers.py:323-327 + model.optimizer.step()
 *                          main.py:203-213 (torch.optim.Adam groups, gaussian_model.py:223-242)
 *   nlosgr_bboxes       <- compute_gaussian_bboxes_kernel include/bbox_compute.cuh:76-120,
 *                          GaussianModel.get_bboxes gaussian_model/gaussian_model.py:140-178
 *   nlosgr_carve_votes  <- the voting loop of space_carving gaussian_model/gaussian_utils.py:88-99
 */
#ifndef NLOSGR_H
#define NLOSGR_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__) || defined(__clang__)
#define NLOSGR_API __attribute__((visibility("default")))
#else
#define NLOSGR_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define NLOSGR_ABI_VERSION 8

/* convention presets */
enum {
    NLOSGR_PRESET_TORCH = 0, /* path T: s=exp(exp(S)*mod), u=R(x-mu), 3DGS SH signs, no eps */
    NLOSGR_PRESET_CUDA = 1   /* path C: s=exp(S)*mod, u=R^T(x-mu)/(s+1e-8), unsigned SH, eps'd normalise */
};

/* per-sample density model */
enum {
    NLOSGR_MODE_NOOCL = 0, /* rho_d = sum_g sigma pdf rho                  (gaussian_model.py:346-364) */
    NLOSGR_MODE_NETF = 1,  /* per-Gaussian self-transmittance cumprod       (gaussian_model.py:313-324) */
    NLOSGR_MODE_BININT = 2, /* no-occlusion with each sample replaced by the exact average of the pdf
                              over its radial bin [r_k -+ dr/2] (closed-form erf; forward only) — the
                              corrected counterpart of the analytic section path */
    NLOSGR_MODE_OCCL = 3   /* path C use_occlusion=True (volume_renderer.cu:80-137), cuda preset only:
                              per ray, T_k = exp(-c dT sum_{k'<k} D_k'), D = sum_g sigma pdf,
                              rho_d = T_k sum_g (1 - exp(-sigma pdf c dT)) rho, zero where T_k < 1e-4 */
};

/* which Gaussians each ray sums over (nlosgr_options.selection) */
enum {
    NLOSGR_SELECT_SUPPORT = 0, /* every Gaussian, samples within the Mahalanobis cutoff (dense if <= 0) */
    NLOSGR_SELECT_AABB = 1     /* path C's filter (ray_aabb.cu:10-61, volume_renderer.cu:220-245): the first
                                  256 Gaussians by index whose 3-sigma box (bbox_compute.cuh) the ray hits,
                                  each evaluated along the whole ray; cuda preset only */
};

enum {
    NLOSGR_OK = 0,
    NLOSGR_E_INVALID = 1, /* bad argument / shape */
    NLOSGR_E_HIP = 2,     /* HIP launch error */
    NLOSGR_E_UNSUPPORTED = 3
};

/* Gaussians: raw (pre-activation) parameters, exactly the reference GaussianModel tensors. */
typedef struct {
    int32_t ng;               /* number of Gaussians */
    int32_t k_feat;           /* feature row stride K >= (sh_degree+1)^2; K <= 25 (torch preset) / 16 (cuda) */
    int32_t sh_degree;        /* active SH degree: 0..4 torch preset (sh_utils.py:57-112), 0..3 cuda preset */
    int32_t preset;           /* NLOSGR_PRESET_* */
    float scaling_modifier;   /* `mod` */
    const float* mu;          /* [ng,3]  _mu                                         */
    const float* scaling;     /* [ng,3]  _scaling (raw)                              */
    const float* rotation;    /* [ng,4]  _rotation (raw quaternion w,x,y,z)          */
    const float* opacity;     /* [ng]    _opacity (raw logit)                        */
    const float* features;    /* [ng,k_feat] cat(_features_dc,_features_rest) flattened */
} nlosgr_gaussians;

/* Batched spherical sampling geometry: one (theta, phi, r) grid per relay-wall point, i.e. the
 * reference's spherical_sample_histogram (nlos_helpers.py:124-188) for P wall points at once.
 * Sample (p, k, i, j) sits at x = wall[p] + r[k] * (st_i cp_j, st_i sp_j, ct_i). */
typedef struct {
    int32_t nwall;            /* P */
    int32_t nt;               /* theta samples (Ns in the reference) */
    int32_t np;               /* phi samples (Ns in the reference) */
    int32_t nr;               /* radial samples = time bins T */
    const float* wall;        /* [P,3] wall points */
    const float* sin_theta;   /* [P,nt] */
    const float* cos_theta;   /* [P,nt] */
    const float* sin_phi;     /* [P,np] */
    const float* cos_phi;     /* [P,np] */
    const float* grid_lin;    /* [P,4] (theta_min, theta_step, phi_min, phi_step) of the linspace grids */
    const float* hscale;      /* [P] histogram weight per wall point (dtheta*dphi*Y^2[*c*dT]) */
    const float* r;           /* [nr] sample radii (linspace, shared by all wall points) */
    const float* att;         /* [nr] per-bin attenuation (1/dist^2 or 1/(t^2+1e-8)) */
} nlosgr_geometry;

typedef struct {
    int32_t mode;             /* NLOSGR_MODE_* */
    float cutoff;             /* Mahalanobis support radius m_c; <= 0 -> dense (no culling) */
    float c_deltaT;           /* c * deltaT (netf transmittance) */
    float ray_scale;          /* scale applied to the optional per-ray output (e.g. c*dT) */
    int32_t nsplit;           /* backward: wall-point splits (0 -> auto) */
    int32_t flags;            /* 0 in production.  Bits 0-6: phase-ablation diagnostics (wrong results on
                                 purpose); NLOSGR_FLAG_* below: variant selection for A/B timing and parity
                                 cross-checks (ABI 8: these used to be environment variables, so the
                                 library's numerics no longer depend on the caller's environment) */
    int32_t ray_cache;        /* 1: the forward records, per (wall point, Gaussian) pair, which rays
                                 of its candidate box are in support (20 B per pair in the workspace,
                                 see nlosgr_workspace_bytes) and a backward on the SAME workspace with
                                 the SAME inputs walks that record instead of re-testing the rays.
                                 Culled (cutoff > 0), histogram-only calls.  In NLOSGR_MODE_OCCL it is
                                 the row cache instead: the forward stores every ray tile's (D, W) rows
                                 (8 B per wall point x ray x bin; C3 128 GiB) and the backward on the
                                 same workspace reloads them instead of re-running its forward sweep
                                 (and, when the forward was one wall-point launch, its tile bins).
                                 0 = off */
    int32_t selection;        /* NLOSGR_SELECT_*.  OCCL mode and AABB selection run the ray-tile engine
                                 (ray-major, per-ray compositing, deterministic); the ray cache and
                                 nlosgr_count_support do not apply there */
    int32_t g_begin, g_end;   /* backward only: gradients of Gaussians [g_begin, g_end) (g_begin % 256 == 0;
                                 rows outside are left untouched), so a caller can all-reduce one
                                 bucket while the next one is differentiated; g_end = 0 -> all */
} nlosgr_options;

/* nlosgr_options.flags: variant selection (each variant is a correct renderer of the same quantity;
 * they differ in summation order / rounding and speed) */
#define NLOSGR_FLAG_FLOAT_DRAIN  0x100  /* forward: fp32 claim drain instead of the fixed-point (FX) drain */
#define NLOSGR_FLAG_MASKED_FWD   0x200  /* forward: masked (end-of-segment) drains at every cutoff, no TAIL */
#define NLOSGR_FLAG_MASKED_BWD   0x400  /* backward: masked drains at every cutoff, no TAIL */
#define NLOSGR_FLAG_LANE_DENSE   0x800  /* dense no-occlusion histogram through the lane-serial drain
                                           instead of the register (lane = bin) kernel */
#define NLOSGR_FLAG_BWD_SHARED   0x1000 /* backward: shared-row layout (4 waves per staged row) */
#define NLOSGR_FLAG_BWD_PERWAVE  0x2000 /* backward: per-wave row layout (default picks by LDS size) */
#define NLOSGR_FLAG_TILE_NOBIN   0x8000 /* ray-tile engine: cull every Gaussian against every item's cone in the
                                           kernel instead of reading the tile bins (A/B: same selections) */
#define NLOSGR_FLAG_FX_MAXUNIT   0x4000 /* forward FX drain: unit from the largest amplitude bound (the round-5
                                           rule, diagnostics: shows the precision the quantile unit recovers) */

/* Scratch bytes needed by fwd/bwd for this problem (caller allocates, 256-B aligned); includes
 * nwall*ng*24 B for the ray cache when opt->ray_cache is set (OCCL mode: the row cache,
 * nwall * tiles * tile rays * nr * 8 B). */
NLOSGR_API size_t nlosgr_workspace_bytes(const nlosgr_gaussians* g, const nlosgr_geometry* geo,
                              const nlosgr_options* opt);

/* Batch budgets in MiB (values <= 0 keep the current one): the backward's dL/drho buffer, filled in
 * wall-point batches (default 1024), and the ray-tile forward's partial histograms (default 1024).
 * (ABI 8: no environment variables are read.)
 * They set the workspace layout: change them only while no workspace sized under the old values is
 * still in use (a ray-cache backward must run under the forward's budgets). */
NLOSGR_API void nlosgr_set_batch_budgets(double drho_mb, double tile_hpart_mb);
/* The batch budgets in effect (MiB): lets a caller restore exactly what it changed. */
NLOSGR_API void nlosgr_get_batch_budgets(double* drho_mb, double* tile_hpart_mb);

/* Forward.  hist_out [P,nr] (may be NULL):  hscale[p]*att[k]*sum_{g,i,j} w_g(p) sin(theta_i) pdf
 *           ray_out  [P,nt*np,nr] (may be NULL, caller zero-fills): ray_scale*sum_g w_g(p) pdf,
 *           rays in the reference's (i,j) meshgrid('ij') order, samples contiguous — the layout of
 *           _C.render_rays' rho_density [N_rays, N_samples].
 * w_g(p) = sigmoid(opacity_g) * max(0, 0.5 + SH_g(dir(mu_g - wall_p))). */
NLOSGR_API int nlosgr_render_fwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo,
                      const nlosgr_options* opt, void* workspace, float* hist_out,
                      float* ray_out, void* hip_stream);

/* Backward.  grad_hist [P,nr] and/or grad_ray [P,nt*np,nr] (either may be NULL).
 * Writes (overwrites) the gradients of the RAW parameters: d_mu [ng,3], d_scaling [ng,3],
 * d_rotation [ng,4], d_opacity [ng], d_features [ng,k_feat]. */
NLOSGR_API int nlosgr_render_bwd(const nlosgr_gaussians* g, const nlosgr_geometry* geo,
                      const nlosgr_options* opt, void* workspace, const float* grad_hist,
                      const float* grad_ray, float* d_mu, float* d_scaling, float* d_rotation,
                      float* d_opacity, float* d_features, void* hip_stream);

/* Work count of one forward at opt->cutoff (no outputs written): counts (DEVICE, [3] uint64,
 * overwritten) = {in-support (wall point, Gaussian) pairs, in-support rays (pair, i, j),
 * in-support evaluations (pair, i, j, k)} — the unit of the VALU roofline. */
NLOSGR_API int nlosgr_count_support(const nlosgr_gaussians* g, const nlosgr_geometry* geo,
                         const nlosgr_options* opt, void* workspace, unsigned long long* counts,
                         void* hip_stream);

/* Fixed-point forward state after an nlosgr_render_fwd on `workspace` (same g / geo / opt): info_out
 * (DEVICE, [4] int32, overwritten, copied on the stream) = {E: the unit 2^-E of the fixed-point drain,
 * E of the launch's largest amplitude bound, LDS histogram flushes into the u64 row, bright segments
 * (peak >= 2^24 units, added straight into the u64 row)}; all zero when the forward did not take the
 * fixed-point drain.  Diagnostics / tests. */
NLOSGR_API int nlosgr_fx_info(const nlosgr_gaussians* g, const nlosgr_geometry* geo, const nlosgr_options* opt,
                   const void* workspace, int32_t* info_out, void* hip_stream);

/* 3-sigma (sigma_scale) axis-aligned boxes [ng,6] = (min xyz, max xyz) under the preset's scale
 * convention (bbox_compute.cuh:23-71 for "cuda"; gaussian_model.py:140-178 for "torch"). */
NLOSGR_API int nlosgr_bboxes(const nlosgr_gaussians* g, float sigma_scale, float* bboxes_out, void* hip_stream);

/* ---------------------------------------------------------------------------------------
 * Path C "rays" API: arbitrary rays x = o + t d (cuda_autograd.py:18-191 -> _C.render_rays,
 * volume_renderer.cu:189-305; _C.filter_gaussians_per_ray, ray_aabb.cu:63-102).
 * ------------------------------------------------------------------------------------- */
#define NLOSGR_MAX_PER_RAY 256   /* MAX_GAUSSIANS_PER_RAY, ray_aabb.cu:6 */

typedef struct nlosgr_rays {
    int32_t nrays;            /* N_rays */
    int32_t nsamp;            /* N_samples (<= 8192) */
    const float* origins;     /* [nrays,3] */
    const float* dirs;        /* [nrays,3], used as given: x = o + t d */
    const float* t;           /* [nsamp] */
    const float* cam;         /* [3] camera position: SH view direction mu - cam */
} nlosgr_rays;

/* Scratch bytes for nlosgr_rays_fwd / nlosgr_rays_bwd. */
NLOSGR_API size_t nlosgr_rays_workspace_bytes(const nlosgr_gaussians* g, const nlosgr_rays* r);

/* filter_out [nrays, 1 + NLOSGR_MAX_PER_RAY] int32: count, then the first (by index) Gaussians
 * whose box bboxes[g] = (min xyz, max xyz) the half-infinite ray hits (slab test with
 * 1/(d + 1e-8), cuda_utils.cuh:97-121), -1 padding — the layout filter_gaussians_per_ray returns. */
NLOSGR_API int nlosgr_filter_rays(const nlosgr_gaussians* g, const nlosgr_rays* r, const float* bboxes,
                       int32_t* filter_out, void* hip_stream);

/* Forward: rho_out, density_out, trans_out [nrays, nsamp] (volume_renderer.cu:16-185):
 *   D = sum_{g in filter} sigmoid(o_g) pdf_g(x);  no occlusion: rho = c dT sum sigma pdf rho_g,
 *   trans = 1;  occlusion: rho = T sum (1 - exp(-sigma pdf c dT)) rho_g, T_s = exp(-c dT
 *   sum_{s'<s} D_s'), all three zero where T_s < 1e-4 (the reference's early exit). */
NLOSGR_API int nlosgr_rays_fwd(const nlosgr_gaussians* g, const nlosgr_rays* r, const int32_t* filter,
                    float c_deltaT, int32_t use_occlusion, void* workspace, float* rho_out,
                    float* density_out, float* trans_out, void* hip_stream);

/* Backward of nlosgr_rays_fwd w.r.t. the RAW parameters (the reference returns zeros,
 * cuda_autograd.py:147-156).  Any of g_rho / g_density / g_trans may be NULL. */
NLOSGR_API int nlosgr_rays_bwd(const nlosgr_gaussians* g, const nlosgr_rays* r, const int32_t* filter,
                    float c_deltaT, int32_t use_occlusion, void* workspace, const float* g_rho,
                    const float* g_density, const float* g_trans, float* d_mu, float* d_scaling,
                    float* d_rotation, float* d_opacity, float* d_features, void* hip_stream);

/* ---------------------------------------------------------------------------------------
 * Path A "analytic section" API (_C.render_rays_analytic, bindings.cpp:6-24,
 * src/volume_renderer_analytic.cu:178-241): hist_out [nrays] = one value per ray.
 * Per ray: the first 128 filter entries whose sigma_threshold-ellipsoid the line o + t d hits,
 * clipped to [t_min, t_max], stably sorted by entry, composited front to back with the
 * reference's closed-form optical depth (analytic_integration.cuh:123-172, formula as written)
 * and early exit at T < 1e-4.  r->t / r->nsamp are unused; features rows have stride k_feat and
 * SH is evaluated to g->sh_degree (unsigned basis, spherical_harmonics.cuh:20-80).  Forward only.
 * ------------------------------------------------------------------------------------- */
NLOSGR_API int nlosgr_rays_analytic(const nlosgr_gaussians* g, const nlosgr_rays* r, const int32_t* filter,
                         float t_min, float t_max, float sigma_threshold, float* hist_out,
                         void* hip_stream);

/* ---------------------------------------------------------------------------------------
 * Fused training step: the loss and the optimizer of the reference's
 * learn_one_iter (main.py:198-254) on the device, with no host synchronisation.
 * ------------------------------------------------------------------------------------- */
#define NLOSGR_ADAM_MAX_GROUPS 8

typedef struct {
    float* param;             /* [n] updated in place */
    const float* grad;        /* [n] */
    float* exp_avg;           /* [n] first-moment state, updated in place (zeros before step 1) */
    float* exp_avg_sq;        /* [n] second-moment state, updated in place */
    long long n;
    double lr;                /* this group's learning rate for this step */
} nlosgr_adam_group;

/* Volume MSE of compute_loss (nlos_helpers.py:323-327) over n elements, target scaled by gt_times:
 * loss_out[4] = {mean((hist - gt*target)^2), loss / mean((gt*target)^2), sum (hist - gt*target)^2,
 * sum (gt*target)^2} (device floats; the raw sums let the ranks of a sharded volume combine exactly);
 * grad_out [n] (may be NULL) = grad_scale * 2 (hist - gt*target) / n.  workspace: caller-owned,
 * nlosgr_mse_workspace_bytes() bytes.  Deterministic (fixed-order reduction, no atomics). */
NLOSGR_API size_t nlosgr_mse_workspace_bytes(void);
NLOSGR_API int nlosgr_mse(const float* hist, const float* target, float gt_times, long long n,
               float grad_scale, float* grad_out, void* workspace, float* loss_out, void* hip_stream);

/* One torch.optim.Adam step (no weight decay, no amsgrad) over 1..NLOSGR_ADAM_MAX_GROUPS parameter
 * groups; `step` >= 1 is the step count including this update (bias correction).  The scalars are
 * doubles so 1 - beta, the bias corrections and lr / (1 - beta1^t) are formed as torch forms them
 * (Python floats) before the fp32 update.  The reference
 * uses betas (0.9, 0.999), eps 1e-15 and six groups (gaussian_model.py:223-242). */
NLOSGR_API int nlosgr_adam(const nlosgr_adam_group* groups, int32_t ngroups, long long step, double beta1,
                double beta2, double eps, void* hip_stream);

/* ---------------------------------------------------------------------------------------
 * Space-carving initialisation.  votes[v] (v < nvox) = number of wall points i
 * with radius[i] > 0 and |coords[v] - walls[i]| >= radius[i] (fp32, torch.norm order, no fma):
 * the voting loop of space_carving (gaussian_utils.py:88-99).  coords [nvox][3], walls [nwall][3]
 * and radius [nwall] are device arrays in the same frame; votes [nvox] int32 is overwritten.
 * ------------------------------------------------------------------------------------- */
NLOSGR_API int nlosgr_carve_votes(const float* coords, long long nvox, const float* walls, const float* radius,
                       int32_t nwall, int32_t* votes, void* hip_stream);

NLOSGR_API const char* nlosgr_last_error(void);
NLOSGR_API int nlosgr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NLOSGR_H */

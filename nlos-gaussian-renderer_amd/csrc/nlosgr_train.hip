// Fused on-device training-step pieces (gfx950): the volume MSE of compute_loss with its
// gradient seed, and the Adam update of the raw Gaussian parameter groups — the per-step host
// work of the reference's learn_one_iter (main.py:198-254: zero_grad, compute_loss, backward,
// optimizer.step) with no host synchronisation.
//
//   mse_kernel   : grad = grad_scale * 2 (hist - gt target) / n, and per-workgroup partial sums
//                  of (hist - gt target)^2 and (gt target)^2; mse_finish_kernel adds the partials
//                  in a fixed order -> loss = mean, equal_loss = loss / mean((gt target)^2)
//                  (nlos_helpers.py:323-327), plus the two raw sums.  Deterministic: no atomics.
//   adam_kernel  : torch.optim.Adam (no weight decay / amsgrad) with per-group learning rates and
//                  the reference's eps = 1e-15 (gaussian_model.py:223-242); grid.y = group, so the
//                  group descriptor is a uniform kernel-argument load.  Op order as torch:
//                  m += (1-b1)(g - m);  v = v b2 + (1-b2) g g;
//                  p += -lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
// Both stream their operands once: HBM-bound, < 1% of a C3 step's time next to the render.
#include "nlosgr_common.hpp"

using namespace nlosgr;
using namespace nlosgr::detail;

namespace {

constexpr int kMseBlocks = 1024;

__global__ __launch_bounds__(kBlock) void mse_kernel(const float* __restrict__ hist, const float* __restrict__ target,
                                                   float gt_times, long long n, float gscale,
                                                   float* __restrict__ grad, float* __restrict__ partial) {
    __shared__ float red[2][kBlock];
    float se = 0.f, st = 0.f;
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock) {
        const float t = target[i] * gt_times;
        const float d = hist[i] - t;
        se = fmaf(d, d, se);
        st = fmaf(t, t, st);
        if (grad) grad[i] = gscale * d;
    }
    red[0][threadIdx.x] = se;
    red[1][threadIdx.x] = st;
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = red[0][0];
        partial[2 * blockIdx.x + 1] = red[1][0];
    }
}

__global__ __launch_bounds__(64) void mse_finish_kernel(const float* __restrict__ partial, int nblk, double n,
                                                      float* __restrict__ out) {
    if (threadIdx.x != 0) return;
    double se = 0.0, st = 0.0;
    for (int b = 0; b < nblk; ++b) {
        se += partial[2 * b];
        st += partial[2 * b + 1];
    }
    const double loss = se / n;
    out[0] = (float)loss;
    out[1] = st > 0.0 ? (float)(loss / (st / n)) : 0.f;
    out[2] = (float)se;   // raw sums: ranks of a sharded volume combine these, not the ratios
    out[3] = (float)st;
}

struct AdamArgs {
    nlosgr_adam_group grp[NLOSGR_ADAM_MAX_GROUPS];
    float b1, b2, omb1, omb2, eps, bc2s;   // 1 - beta formed in double (torch's scalar arithmetic)
    float step_size[NLOSGR_ADAM_MAX_GROUPS];   // lr / (1 - b1^t), formed in double
};

__global__ __launch_bounds__(kBlock) void adam_kernel(AdamArgs a) {
    const nlosgr_adam_group& G = a.grp[blockIdx.y];
    const float ss = a.step_size[blockIdx.y];
    for (long long j = blockIdx.x * (long long)kBlock + threadIdx.x; j < G.n; j += (long long)gridDim.x * kBlock) {
        const float g = G.grad[j];
        float m = G.exp_avg[j];
        m = m + a.omb1 * (g - m);                   // exp_avg.lerp_(grad, 1 - beta1)
        float v = G.exp_avg_sq[j] * a.b2;                  // exp_avg_sq.mul_(beta2)
        v = v + a.omb2 * (g * g);                     //           .addcmul_(grad, grad, 1 - beta2)
        G.exp_avg[j] = m;
        G.exp_avg_sq[j] = v;
        const float denom = sqrtf(v) / a.bc2s + a.eps;     // (sqrt(v) / sqrt(bc2)).add_(eps)
        G.param[j] = G.param[j] + (-ss) * (m / denom);     // param.addcdiv_(m, denom, -step_size)
    }
}

}  // namespace

extern "C" {

size_t nlosgr_mse_workspace_bytes(void) { return (size_t)2 * kMseBlocks * sizeof(float); }

int nlosgr_mse(const float* hist, const float* target, float gt_times, long long n, float grad_scale,
               float* grad_out, void* workspace, float* loss_out, void* hip_stream) {
    if (n < 0) return set_err(NLOSGR_E_INVALID, "n must be >= 0");
    if (!loss_out || !workspace) return set_err(NLOSGR_E_INVALID, "null loss/workspace pointer");
    if (n > 0 && (!hist || !target)) return set_err(NLOSGR_E_INVALID, "null hist/target pointer");
    hipStream_t s = (hipStream_t)hip_stream;
    const long long want = (n + kBlock - 1) / kBlock;
    const int nblk = (int)(want < kMseBlocks ? (want > 0 ? want : 1) : kMseBlocks);
    const float gscale = n > 0 ? (float)((double)grad_scale * 2.0 / (double)n) : 0.f;
    hipLaunchKernelGGL(mse_kernel, dim3(nblk), dim3(kBlock), 0, s, hist, target, gt_times, n, gscale, grad_out,
                       (float*)workspace);
    hipLaunchKernelGGL(mse_finish_kernel, dim3(1), dim3(64), 0, s, (const float*)workspace, nblk,
                       (double)(n > 0 ? n : 1), loss_out);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

int nlosgr_adam(const nlosgr_adam_group* groups, int32_t ngroups, long long step, double beta1, double beta2,
                double eps, void* hip_stream) {
    if (!groups || ngroups < 1 || ngroups > NLOSGR_ADAM_MAX_GROUPS)
        return set_err(NLOSGR_E_INVALID, "1 <= ngroups <= NLOSGR_ADAM_MAX_GROUPS");
    if (step < 1) return set_err(NLOSGR_E_INVALID, "step must be >= 1");
    AdamArgs a;
    memset(&a, 0, sizeof(a));
    long long nmax = 0;
    const double bc1 = 1.0 - pow(beta1, (double)step);
    for (int g = 0; g < ngroups; ++g) {
        const nlosgr_adam_group& G = groups[g];
        if (G.n < 0) return set_err(NLOSGR_E_INVALID, "group size must be >= 0");
        if (G.n > 0 && (!G.param || !G.grad || !G.exp_avg || !G.exp_avg_sq))
            return set_err(NLOSGR_E_INVALID, "null Adam group pointer");
        a.grp[g] = G;
        a.step_size[g] = (float)(G.lr / bc1);
        if (G.n > nmax) nmax = G.n;
    }
    a.b1 = (float)beta1; a.b2 = (float)beta2; a.eps = (float)eps;
    a.omb1 = (float)(1.0 - beta1);
    a.omb2 = (float)(1.0 - beta2);
    a.bc2s = (float)sqrt(1.0 - pow(beta2, (double)step));
    if (nmax == 0) return NLOSGR_OK;
    const long long want = (nmax + kBlock - 1) / kBlock;
    const int nblk = (int)(want < 1024 ? want : 1024);
    hipLaunchKernelGGL(adam_kernel, dim3(nblk, ngroups), dim3(kBlock), 0, (hipStream_t)hip_stream, a);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

}  // extern "C"

// Space-carving initialisation (gfx950), SURVEY §8f rank 4: the voting loop of the reference's
// space_carving (gaussian_model/gaussian_utils.py:88-99).  For every voxel v of the carving grid,
//     votes[v] = #{ wall points i : radius[i] > 0 and |coords[v] - walls[i]| >= radius[i] }
// i.e. the number of first-bounce spheres the voxel lies outside of.  The reference runs one
// torch pass over all voxels per wall point from Python (O(M*N) with M*N host iterations); here
// lane = voxel and the wall points stream through LDS in tiles of 256, so one launch does the lot.
// Distances follow torch.norm in fp32 without contraction: sqrt((dx*dx + dy*dy) + dz*dz).
#include "nlosgr_common.hpp"

using namespace nlosgr;
using namespace nlosgr::detail;

namespace {

constexpr int kCarveTile = 256;

__global__ __launch_bounds__(kBlock) void carve_kernel(const float* __restrict__ coords, long long nvox,
                                                       const float* __restrict__ walls,
                                                       const float* __restrict__ radius, int nwall,
                                                       int32_t* __restrict__ votes) {
    __shared__ float4 tile[kCarveTile];
    const long long v = (long long)blockIdx.x * kBlock + threadIdx.x;
    const bool live = v < nvox;
    const float x = live ? coords[3 * v] : 0.f, y = live ? coords[3 * v + 1] : 0.f, z = live ? coords[3 * v + 2] : 0.f;
    int cnt = 0;
    for (int base = 0; base < nwall; base += kCarveTile) {
        __syncthreads();
        const int i = base + (int)threadIdx.x;
        tile[threadIdx.x] = i < nwall ? make_float4(walls[3 * i], walls[3 * i + 1], walls[3 * i + 2], radius[i])
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
        const int n = min(kCarveTile, nwall - base);
        for (int j = 0; j < n; ++j) {
            const float4 t = tile[j];
            const float dx = __fsub_rn(x, t.x), dy = __fsub_rn(y, t.y), dz = __fsub_rn(z, t.z);
            const float d = sqrtf(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
            cnt += (t.w > 0.f && !(d < t.w)) ? 1 : 0;
        }
    }
    if (live) votes[v] = cnt;
}

}  // namespace

extern "C" {

int nlosgr_carve_votes(const float* coords, long long nvox, const float* walls, const float* radius, int32_t nwall,
                       int32_t* votes, void* hip_stream) {
    if (nvox < 0 || nwall < 0) return set_err(NLOSGR_E_INVALID, "nvox and nwall must be >= 0");
    if (nvox == 0) return NLOSGR_OK;
    if (!coords || !votes || (nwall > 0 && (!walls || !radius)))
        return set_err(NLOSGR_E_INVALID, "null carving pointer");
    const long long nb = (nvox + kBlock - 1) / kBlock;
    if (nb > 0x7FFFFFFFll) return set_err(NLOSGR_E_INVALID, "carving grid too large");
    hipLaunchKernelGGL(carve_kernel, dim3((unsigned)nb), dim3(kBlock), 0, (hipStream_t)hip_stream, coords, nvox, walls,
                       radius, (int)nwall, votes);
    HIPCHK(hipGetLastError());
    return NLOSGR_OK;
}

}  // extern "C"

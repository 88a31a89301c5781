// ds_permute_b32 semantics on gfx950 (collisions, unwritten lanes, inactive lanes): one wave, prints
// the value each lane receives.  hipcc --offload-arch=gfx950 -O2 scripts/permute_probe.hip -o /tmp/pp
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void probe(int* out) {
    const int lane = threadIdx.x;
    int r = -1;
    if (lane % 3 != 2) {   // lanes 2, 5, 8, ... inactive
        const int dst = (lane * 7) % 5;          // destinations 0..4 only, with collisions
        r = __builtin_amdgcn_ds_permute(dst * 4, lane + 100);
    }
    out[lane] = r;
    // second probe: all lanes active, every lane sends to lane 0 or 1
    const int r2 = __builtin_amdgcn_ds_permute((lane & 1) * 4, lane + 1000);
    out[64 + lane] = r2;
}
int main() {
    int* d; int h[128];
    hipMalloc(&d, 128 * sizeof(int));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("probe1 (lane: value):");
    for (int i = 0; i < 64; ++i) printf(" %d:%d", i, h[i]);
    printf("\nprobe2:");
    for (int i = 0; i < 8; ++i) printf(" %d:%d", i, h[64 + i]);
    printf("\n");
    return 0;
}

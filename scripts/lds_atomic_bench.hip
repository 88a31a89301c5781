// Microbenchmark (diagnostic, not product): cost of scatter-adding one value per lane per step into
// a wave's LDS histogram on gfx950, for the forward drain's choice of accumulation primitive.
//   mode 0: ds_read_b32 -> v_add_f32 -> ds_write_b32 chain (the current drain; one LDS round trip per step)
//   mode 1: ds_add_u32  (no return)
//   mode 2: ds_add_u64  (no return)
//   mode 3: ds_add_f32  (no return)
//   mode 4: ds_add_u64 into ONE workgroup-shared histogram (4 waves add to the same bins)
//   modes 5/6/7: as 0/1/2 with bank-conflict-free positions (lane l starts at a wave base + l)
//   mode 8/9: read-add-write chain of float2 / float4 (2 / 4 bins per LDS op) at random aligned starts;
//             reported per BIN-step (16 bins per lane per iteration in every mode)
// Each lane owns a start bin (distinct per wave, pseudo-random) and adds at start + m, m = 0..15.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kBins = 1024, kSteps = 16, kIters = 2000, kBlocks = 256 * 8;

template <int MODE0>
__global__ __launch_bounds__(256) void bench(float* out, int seed) {
    constexpr int MODE = MODE0 >= 8 ? MODE0 : (MODE0 >= 5 ? MODE0 - 5 : MODE0);
    constexpr bool CF = MODE0 >= 5 && MODE0 < 8;
    constexpr int W = (MODE == 2 || MODE == 4) ? 2 : 1;   // words per bin
    __shared__ __align__(16) unsigned h32[W * 4 * (kBins + 64)];
    unsigned long long* h64 = reinterpret_cast<unsigned long long*>(h32);
    float* hf = reinterpret_cast<float*>(h32);
    unsigned* hu = h32;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int t = threadIdx.x; t < W * 4 * (kBins + 64); t += 256) h32[t] = 0u;
    __syncthreads();
    unsigned st = (unsigned)(lane * 2654435761u) ^ (unsigned)(seed + blockIdx.x);
    float v = 1.0f + lane * 1e-3f;
    const int wbase = (MODE == 4) ? 0 : wave * (kBins + 64);
    for (int it = 0; it < kIters; ++it) {
        st = st * 1664525u + 1013904223u;
        const int pos = CF ? (int)(__builtin_amdgcn_readfirstlane((st >> 8) % (kBins - kSteps - 64)) + lane)
                           : (int)((st >> 8) % (kBins - kSteps));
        if (MODE == 8) {
            float2* hb = reinterpret_cast<float2*>(hf + wbase + (pos & ~1));
#pragma unroll
            for (int m = 0; m < kSteps / 2; ++m) {
                float2 x = hb[m];
                x.x += v; x.y += v;
                hb[m] = x;
                __asm__ __volatile__("" ::: "memory");
            }
        } else if (MODE == 9) {
            float4* hb = reinterpret_cast<float4*>(hf + wbase + (pos & ~3));
#pragma unroll
            for (int m = 0; m < kSteps / 4; ++m) {
                float4 x = hb[m];
                x.x += v; x.y += v; x.z += v; x.w += v;
                hb[m] = x;
                __asm__ __volatile__("" ::: "memory");
            }
        } else if (MODE == 0) {
            float* hb = hf + wbase + pos;
#pragma unroll
            for (int m = 0; m < kSteps; ++m) {
                const float x = hb[m];
                hb[m] = x + v;
                __asm__ __volatile__("" ::: "memory");
            }
        } else if (MODE == 1) {
#pragma unroll
            for (int m = 0; m < kSteps; ++m) __hip_atomic_fetch_add(hu + wbase + pos + m, (unsigned)(v * 1000.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (MODE == 2 || MODE == 4) {
#pragma unroll
            for (int m = 0; m < kSteps; ++m) __hip_atomic_fetch_add(h64 + wbase + pos + m, (unsigned long long)(unsigned)(v * 1000.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
#pragma unroll
            for (int m = 0; m < kSteps; ++m) __hip_atomic_fetch_add(hf + wbase + pos + m, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        v = v * 1.0001f;
    }
    __syncthreads();
    float s = 0.f;
    for (int t = threadIdx.x; t < W * 4 * (kBins + 64); t += 256) s += (float)(h32[t] & 0xffff);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
float run(float* d) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    bench<MODE><<<kBlocks, 256>>>(d, 1);
    hipEventRecord(a);
    bench<MODE><<<kBlocks, 256>>>(d, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    // LDS ops per CU per cycle (2.4 GHz, 256 CUs): wave-instructions
    const double winst = (double)kBlocks * 4 * kIters * kSteps;
    printf("mode %d: %.3f ms  %.2f cycles per wave-step per CU\n", MODE, ms, ms * 1e-3 * 2.4e9 * 256 / winst);
    return ms;
}

int main() {
    float* d;
    hipMalloc(&d, kBlocks * 256 * sizeof(float));
    run<0>(d); run<1>(d); run<2>(d); run<3>(d); run<4>(d); run<5>(d); run<6>(d); run<7>(d); run<8>(d); run<9>(d);
    hipFree(d);
    return 0;
}

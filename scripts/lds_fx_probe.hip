// Microbenchmark (diagnostic, not product): the forward drain's scatter-add into a wave's LDS
// histogram, float2 read-add-write (the claim drain's access) against packed fixed-point
// ds_add_u64 (two 32-bit bin fields per 64-bit word, no claims), at random and at clustered start
// bins (the real drain's segments of one wave start near each other).  Reported per BIN.
//   mode 0: float2 read-add-write, random even starts          (2 bins per op pair)
//   mode 1: ds_add_u64 packed, random even starts              (2 bins per op)
//   mode 2: float2 read-add-write, starts within 48 bins of a wave base
//   mode 3: ds_add_u64 packed, starts within 48 bins of a wave base
//   mode 4: ds_add_u64 packed, starts within 12 bins of a wave base (heavy clustering)
//   mode 5: float2 read-add-write, starts within 12 bins of a wave base
//   mode 6: ds_add_u64 packed, distinct consecutive pairs (lane l at base + 2l: conflict-free)
//   mode 7: as mode 1 with only lanes 0-31 active (does a masked lane cost LDS cycles?)
//   mode 8: as mode 1 with every other lane active (32 active, all four 16-lane groups busy)
//   mode 9: as mode 6 with lanes 0-31 active
//   mode 10: ds_add_f32 (no return) at random bins, one bin per op (build with -munsafe-fp-atomics)
//   mode 11: ds_add_u64, lane l at word base + (l mod 16) + 32 (l / 16): distinct mod 16 within each
//            16-lane group, lanes l and l + 16 on the same word mod 32 (which lane grouping banks it?)
//   mode 12: ds_add_u64, lane l at word base + (l mod 32) + 64 (l / 32): distinct mod 32 within each half
//   mode 13: ds_add_u64, lane l at word base + 16 (l mod 4) + (l / 4): 16-lane groups hold 4 runs of 4
//   mode 14: ds_add_u64, lane l at word base + 2 (l mod 16) + 64 (l / 16): 2-way mod 16, distinct mod 32 per group
//   mode 15: ds_add_u64, lane l at word base + (l mod 16) + 16 (l / 16) + 48 (l / 32): groups of 16 distinct
//            mod 16; lanes l and l + 16 distinct mod 32; lanes l and l + 32 equal mod 64 words
//   mode 16: ds_add_u64, lane l at word base + 16 l: all 64 lanes on one word residue mod 16 (16-way per group)
//   mode 17: ds_add_u64, lane l at word base + (l mod 16) + (l / 16): conflict-free within each group, but the
//            groups' words overlap (lane l of group g and lane l + 1 of group g - 1 share an address)
//   mode 18: ds_add_u64, lane l at word base + (l mod 16): the 4 groups on the same 16 addresses
//   mode 19: ds_add_u64, lane l at word base + (l mod 16) + 16 (l / 16) - (l / 16): as 17 with groups 15 words apart
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ unsigned cvt_rpi(float x) {   // floor(x + 0.5) as an integer, one VALU op
    int r;
    __asm__("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return (unsigned)r;
}

constexpr int kBins = 1024, kSteps = 20, kIters = 2000, kBlocks = 256 * 12;

template <int MODE>
__global__ __launch_bounds__(256) void bench(float* out, int seed) {
    constexpr bool ATOM = MODE == 1 || MODE == 3 || MODE == 4 || (MODE >= 6 && MODE != 10);
    constexpr bool PATTERN = MODE >= 11;
    constexpr int SPREAD = (MODE == 2 || MODE == 3) ? 48 : ((MODE == 4 || MODE == 5) ? 12 : 0);
    __shared__ __align__(16) unsigned h32[4 * (kBins + 640)];
    for (int t = threadIdx.x; t < 4 * (kBins + 640); t += 256) h32[t] = 0u;
    (void)PATTERN;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned st = (unsigned)(lane * 2654435761u) ^ (unsigned)(seed + blockIdx.x * 7919);
    float v = 1.0f + lane * 1e-3f;
    const int wbase = wave * (kBins + 640);
    for (int it = 0; it < kIters; ++it) {
        st = st * 1664525u + 1013904223u;
        int pos;
        if (PATTERN) {
            const int b = (int)(__builtin_amdgcn_readfirstlane((st >> 8) % (kBins - 300)) & ~1);
            const int w = MODE == 11 ? (lane % 16) + 32 * (lane / 16)
                        : MODE == 12 ? (lane % 32) + 64 * (lane / 32)
                        : MODE == 13 ? 16 * (lane % 4) + lane / 4
                        : MODE == 14 ? 2 * (lane % 16) + 64 * (lane / 16)
                        : MODE == 15 ? (lane % 16) + 16 * (lane / 16) + 48 * (lane / 32)
                        : MODE == 17 ? (lane % 16) + (lane / 16)
                        : MODE == 18 ? (lane % 16)
                        : MODE == 19 ? (lane % 16) + 15 * (lane / 16) : 16 * lane;
            pos = b + 2 * (w % 256);
        } else if (MODE == 6 || MODE == 9) {
            pos = (int)(__builtin_amdgcn_readfirstlane((st >> 8) % (kBins - 160)) & ~1) + 2 * lane;
        } else if (SPREAD) {
            const unsigned b = __builtin_amdgcn_readfirstlane((st >> 8) % (kBins - kSteps - SPREAD));
            pos = (int)(b + ((st >> 20) % SPREAD)) & ~1;
        } else {
            pos = (int)((st >> 8) % (kBins - kSteps)) & ~1;
        }
        if (MODE == 10) {
            float* hf = reinterpret_cast<float*>(h32) + wbase + pos;
#pragma unroll
            for (int m = 0; m < kSteps / 2; ++m)
                __hip_atomic_fetch_add(hf + 2 * m, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (!ATOM) {
            float2* hb = reinterpret_cast<float2*>(reinterpret_cast<float*>(h32) + wbase + pos);
#pragma unroll
            for (int m = 0; m < kSteps / 2; ++m) {
                float2 x = hb[m];
                x.x += v; x.y += v * 0.5f;
                hb[m] = x;
                __asm__ __volatile__("" ::: "memory");
            }
        } else if ((MODE == 7 || MODE == 9) && lane >= 32) {
        } else if (MODE == 8 && (lane & 1)) {
        } else {
            unsigned long long* hb = reinterpret_cast<unsigned long long*>(h32 + wbase + pos);
#pragma unroll
            for (int m = 0; m < kSteps / 2; ++m) {
                const unsigned lo = (unsigned)cvt_rpi((float)m * v), hi = (unsigned)cvt_rpi(v);
                __hip_atomic_fetch_add(hb + m, ((unsigned long long)hi << 32) | lo, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        v = v * 1.0001f;
    }
    __syncthreads();
    float s = 0.f;
    for (int t = threadIdx.x; t < 4 * (kBins + 640); t += 256) s += (float)(h32[t] & 0xffff);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(float* d) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    bench<MODE><<<kBlocks, 256>>>(d, 1);
    hipEventRecord(a);
    bench<MODE><<<kBlocks, 256>>>(d, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double bins = (double)kBlocks * 4 * kIters * kSteps;   // wave bin-steps
    printf("mode %d: %.3f ms  %.2f CU-cycles per wave bin-step (2.4 GHz, 256 CUs)\n", MODE, ms,
           ms * 1e-3 * 2.4e9 * 256 / bins);
}

int main() {
    float* d;
    hipMalloc(&d, kBlocks * 256 * sizeof(float));
    run<0>(d); run<1>(d); run<2>(d); run<3>(d); run<4>(d); run<5>(d); run<6>(d); run<7>(d); run<8>(d); run<9>(d); run<10>(d); run<11>(d); run<12>(d); run<13>(d); run<14>(d); run<15>(d); run<16>(d); run<17>(d); run<18>(d); run<19>(d);
    hipFree(d);
    return 0;
}

// Microbenchmark (diagnostic, not product): candidate no-occlusion forward drains on gfx950, fed with
// synthetic ray segments shaped like C3's at 5.7 sigma (length 98 sqrt(1-u) bins x exp(0.2 N), random
// start in a 1024-bin histogram).  Reports CU-cycles per 64 useful (in-segment) bin evaluations; the
// production lane-serial claim drain runs at ~13 on C3 (890 ms for 2.69e12 evaluations).
//   V0 VALU rates: v_fma_f32 / v_exp_f32 / v_mul_f32 chains (cycles per wave-instruction per SIMD)
//   V1 half-wave per segment, 2 bins per lane, exp2 per bin, ds_read_b64/ds_write_b64 into a
//      histogram private to the half (no claims)
//   V2 half-wave per segment, 1 bin per lane, b32 read-add-write
//   V3 quarter-wave per segment, 2 bins per lane, 4 private histograms per wave
//   V4 lane = bin, (segment, 64-bin block) items pre-bucketed by block, register accumulator
//      flushed once per bucket; item records read with wave-uniform (scalar) loads
//   V5 as V4 with 32-bin blocks and two items per step (one per half-wave)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <string.h>

constexpr int kNR = 1024, kPadH = 1024 + 128;
constexpr int kSeg = 256;          // segments per wave
constexpr int kRep = 40;           // passes over a wave's segments
constexpr int kWG = 2048;          // workgroups (4 waves)
constexpr float kHL2E = 0.72134752044448170368f;

struct Seg { float ga, al, ks; int kl, len; };
static float hbits(int x) { float f; memcpy(&f, &x, 4); return f; }

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int OP>
__global__ __launch_bounds__(256) void valu_rate(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = s + 1e-3f * (threadIdx.x + i);
    for (int it = 0; it < 4096; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) a[i] = fmaf(a[i], 0.999f, 1e-4f);
            else if (OP == 1) a[i] = ex2(a[i]) * -0.5f;   // exp + mul (the mul is counted separately by OP 2)
            else a[i] = a[i] * 0.9999f;
        }
    }
    float t = 0.f;
    for (int i = 0; i < 8; ++i) t += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

// segment records float4 (ga, al, t0 = kl - ks, kl | len << 16)
template <int GROUP, int BPL>   // lanes per segment, bins per lane
__global__ __launch_bounds__(256) void drain_seg(const float4* __restrict__ recs, float* out) {
    constexpr int NG = 64 / GROUP;           // segment groups per wave (private histograms)
    constexpr int SPAN = GROUP * BPL;        // bins per step
    extern __shared__ __align__(16) float sm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int grp = lane / GROUP, gl = lane % GROUP;
    float4* rq = reinterpret_cast<float4*>(sm) + wave * kSeg;
    float* hist = sm + 4 * 4 * kSeg + (wave * NG + grp) * kPadH;
    const float4* src = recs + ((size_t)blockIdx.x * 4 + wave) * kSeg;
    for (int i = lane; i < kSeg; i += 64) rq[i] = src[i];
    for (int i = gl; i < kPadH; i += GROUP) hist[i] = 0.f;
    __syncthreads();
    for (int rep = 0; rep < kRep; ++rep) {
        int idx = grp;                   // this group's next segment
        float4 r = rq[idx];
        int pos = __float_as_int(r.w) & 0xFFFF, rem = __float_as_int(r.w) >> 16;
        float t = r.z + (float)(BPL * gl);
        if (BPL == 2) { t -= (float)(pos & 1); rem += pos & 1; pos &= ~1; }
        while (true) {
            const bool live = idx < kSeg;
            if (!__builtin_amdgcn_ballot_w64(live)) break;
            if (live) {
                if (BPL == 2) {
                    float2* hb = reinterpret_cast<float2*>(hist + pos) + gl;
                    const float v0 = ex2(fmaf(r.x, t * t, r.y));
                    const float t1 = t + 1.f;
                    const float v1 = ex2(fmaf(r.x, t1 * t1, r.y));
                    float2 x = *hb;
                    x.x += v0; x.y += v1;
                    *hb = x;
                } else {
                    float* hb = hist + pos + gl;
                    const float v0 = ex2(fmaf(r.x, t * t, r.y));
                    *hb += v0;
                }
                pos += SPAN; rem -= SPAN; t += (float)SPAN;
                if (rem <= 0) {
                    idx += NG;
                    r = rq[min(idx, kSeg - 1)];
                    pos = __float_as_int(r.w) & 0xFFFF; rem = __float_as_int(r.w) >> 16;
                    t = r.z + (float)(BPL * gl);
                    if (BPL == 2) { t -= (float)(pos & 1); rem += pos & 1; pos &= ~1; }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    float s = 0.f;
    for (int i = gl; i < kPadH; i += GROUP) s += hist[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// item lists per wave: bucket offsets [nb + 1] then items (float4 ga, al, ks - block base, unused)
template <int BW>
__global__ __launch_bounds__(256) void drain_reg(const float4* __restrict__ items, const int* __restrict__ boff,
                                                 int nb, int per_wave, float* out) {
    __shared__ float hist[4][kPadH];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wid = blockIdx.x * 4 + wave;
    const float4* it = items + (size_t)wid * per_wave;
    const int* bo = boff + (size_t)wid * (nb + 1);
    for (int i = lane; i < kPadH; i += 64) hist[wave][i] = 0.f;
    __syncthreads();
    constexpr int H = 64 / BW;   // items per step (lane groups)
    const int sub = lane / BW, L = lane % BW;
    const float fl = (float)L;
    for (int rep = 0; rep < kRep; ++rep) {
        for (int b = 0; b < nb; ++b) {
            const int i0 = __builtin_amdgcn_readfirstlane(bo[b]), i1 = __builtin_amdgcn_readfirstlane(bo[b + 1]);
            if (i0 == i1) continue;
            float acc = 0.f;
            for (int i = i0; i < i1; i += H) {
                float4 e;
                if (H == 1) {
                    e = it[i];
                } else {
                    const float4 e0 = it[i], e1 = it[min(i + 1, i1 - 1)];
                    const bool ok1 = i + 1 < i1;
                    e.x = sub ? e1.x : e0.x;
                    e.y = sub ? (ok1 ? e1.y : -1e30f) : e0.y;
                    e.z = sub ? e1.z : e0.z;
                }
                const float t = fl - e.z;
                acc += ex2(fmaf(e.x, t * t, e.y));
            }
            if (H > 1) acc += __shfl_xor(acc, 32);
            if (lane < BW) hist[wave][b * BW + L] += acc;
        }
    }
    __syncthreads();
    float s = 0.f;
    for (int i = lane; i < kPadH; i += 64) s += hist[wave][i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

static float timeit(void (*launch)(void*), void* arg) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch(arg);
    hipDeviceSynchronize();
    hipEventRecord(a);
    launch(arg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = -1.f;
    hipError_t e = hipEventElapsedTime(&ms, a, b);
    hipError_t le = hipGetLastError();
    if (e != hipSuccess || le != hipSuccess) printf("hip error: %s / %s\n", hipGetErrorString(e), hipGetErrorString(le));
    return ms;
}

struct Ctx { float* out; float4* recs; float4* items; int* boff; int nb; int per_wave; };

int main() {
    int ndev = 0; hipError_t de = hipGetDeviceCount(&ndev); printf("devices %d (%s)\n", ndev, hipGetErrorString(de));
    // synthetic segments
    srand(7);
    auto urand = []() { return (rand() + 0.5) / ((double)RAND_MAX + 1.0); };
    const size_t nseg = (size_t)kWG * 4 * kSeg;
    std::vector<Seg> segs(nseg);
    double useful = 0;
    const float mc2 = 5.7f * 5.7f;
    for (auto& s : segs) {
        const double u = urand();
        const double g = exp(0.2 * sqrt(-2 * log(urand())) * cos(6.283185307 * urand()));
        int len = (int)(98.0 * g * sqrt(1 - u));
        len = std::max(1, std::min(len, 400));
        const int kl = (int)(urand() * (kNR - len));
        const double h = 0.5 * len + 0.5;
        s.kl = kl; s.len = len; s.ks = kl + 0.5f * (len - 1);
        s.ga = -kHL2E * mc2 * (float)(1 - u) / (float)(h * h);
        s.al = -kHL2E * mc2 * (float)u;
        useful += len;
    }
    useful *= kRep;
    std::vector<float4> recs(nseg);
    for (size_t i = 0; i < nseg; ++i) {
        const Seg& s = segs[i];
        recs[i] = make_float4(s.ga, s.al, (float)s.kl - s.ks, hbits(s.kl | (s.len << 16)));
    }
    Ctx c;
    hipMalloc(&c.out, (size_t)4096 * 256 * 4);   // V0 launches 4096 blocks
    hipFuncSetAttribute((const void*)drain_seg<32, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)drain_seg<32, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)drain_seg<16, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipMalloc(&c.recs, nseg * sizeof(float4));
    hipMemcpy(c.recs, recs.data(), nseg * sizeof(float4), hipMemcpyHostToDevice);
    const double cu_cyc = 2.4e9 * 256 * 1e-3;   // CU-cycles per ms

    // V0
    {
        auto l0 = [](void* a) { valu_rate<0><<<4096, 256>>>(((Ctx*)a)->out, 1.f); };
        auto l1 = [](void* a) { valu_rate<1><<<4096, 256>>>(((Ctx*)a)->out, 1.f); };
        auto l2 = [](void* a) { valu_rate<2><<<4096, 256>>>(((Ctx*)a)->out, 1.f); };
        const double winst = 4096.0 * 4 * 4096 * 8;   // wave-instructions
        const double simd = 2.4e9 * 256 * 4 * 1e-3;    // SIMD-cycles per ms
        float m0 = timeit(l0, &c), m1 = timeit(l1, &c), m2 = timeit(l2, &c);
        printf("V0 fma %.2f  exp+mul %.2f  mul %.2f  -> exp alone %.2f SIMD-cycles per wave-instruction\n",
               m0 * simd / winst, m1 * simd / winst, m2 * simd / winst, (m1 - m2) * simd / winst);
    }
    {
        const size_t sm = 4 * 4 * kSeg * 4 + 4 * 2 * kPadH * 4;
        auto l = [](void* a) {
            Ctx* c = (Ctx*)a;
            drain_seg<32, 2><<<kWG, 256, 4 * 4 * kSeg * 4 + 4 * 2 * kPadH * 4>>>(c->recs, c->out);
        };
        (void)sm;
        float ms = timeit(l, &c);
        printf("V1 half-wave 2 bins/lane: %.3f ms  %.2f CU-cycles per 64 useful\n", ms, ms * cu_cyc / (useful / 64));
    }
    {
        auto l = [](void* a) {
            Ctx* c = (Ctx*)a;
            drain_seg<32, 1><<<kWG, 256, 4 * 4 * kSeg * 4 + 4 * 2 * kPadH * 4>>>(c->recs, c->out);
        };
        float ms = timeit(l, &c);
        printf("V2 half-wave 1 bin/lane:  %.3f ms  %.2f CU-cycles per 64 useful\n", ms, ms * cu_cyc / (useful / 64));
    }
    {
        auto l = [](void* a) {
            Ctx* c = (Ctx*)a;
            drain_seg<16, 2><<<kWG, 256, 4 * 4 * kSeg * 4 + 4 * 4 * kPadH * 4>>>(c->recs, c->out);
        };
        float ms = timeit(l, &c);
        printf("V3 quarter 2 bins/lane:   %.3f ms  %.2f CU-cycles per 64 useful\n", ms, ms * cu_cyc / (useful / 64));
    }
    for (int BW : {64, 32}) {
        // bucket items by BW-bin block per wave
        const int nb = kNR / BW;
        std::vector<std::vector<float4>> per(kWG * 4);
        size_t maxn = 0;
        for (int w = 0; w < kWG * 4; ++w) {
            std::vector<std::vector<float4>> bk(nb);
            for (int i = 0; i < kSeg; ++i) {
                const Seg& s = segs[(size_t)w * kSeg + i];
                for (int b = s.kl / BW; b <= (s.kl + s.len - 1) / BW; ++b)
                    bk[b].push_back(make_float4(s.ga, s.al, s.ks - (float)(b * BW), 0.f));
            }
            for (auto& v : bk) per[w].insert(per[w].end(), v.begin(), v.end());
            maxn = std::max(maxn, per[w].size());
        }
        std::vector<float4> items(maxn * kWG * 4);
        std::vector<int> boff((size_t)(nb + 1) * kWG * 4);
        for (int w = 0; w < kWG * 4; ++w) {
            std::vector<int> cnt(nb, 0);
            for (int i = 0; i < kSeg; ++i) {
                const Seg& s = segs[(size_t)w * kSeg + i];
                for (int b = s.kl / BW; b <= (s.kl + s.len - 1) / BW; ++b) cnt[b]++;
            }
            int o = 0;
            for (int b = 0; b < nb; ++b) { boff[(size_t)w * (nb + 1) + b] = o; o += cnt[b]; }
            boff[(size_t)w * (nb + 1) + nb] = o;
            std::copy(per[w].begin(), per[w].end(), items.begin() + (size_t)w * maxn);
        }
        hipMalloc(&c.items, items.size() * sizeof(float4));
        hipMalloc(&c.boff, boff.size() * sizeof(int));
        hipMemcpy(c.items, items.data(), items.size() * sizeof(float4), hipMemcpyHostToDevice);
        hipMemcpy(c.boff, boff.data(), boff.size() * sizeof(int), hipMemcpyHostToDevice);
        c.nb = nb; c.per_wave = (int)maxn;
        float ms;
        if (BW == 64) {
            auto l = [](void* a) { Ctx* c = (Ctx*)a; drain_reg<64><<<kWG, 256>>>(c->items, c->boff, c->nb, c->per_wave, c->out); };
            ms = timeit(l, &c);
        } else {
            auto l = [](void* a) { Ctx* c = (Ctx*)a; drain_reg<32><<<kWG, 256>>>(c->items, c->boff, c->nb, c->per_wave, c->out); };
            ms = timeit(l, &c);
        }
        printf("V%d lane=bin, %d-bin items: %.3f ms  %.2f CU-cycles per 64 useful\n", BW == 64 ? 4 : 5, BW, ms,
               ms * cu_cyc / (useful / 64));
        hipFree(c.items); hipFree(c.boff);
    }
    return 0;
}

// Microbenchmark (diagnostic, not product): fixed-point forward drains on gfx950, fed with synthetic ray
// segments shaped like C3's at 5.7 sigma (scripts/drain_proto.hip's distribution: length 98 sqrt(1-u) bins x
// exp(0.2 N), random start in a 1024-bin histogram), every value added as a packed pair of 32-bit units
// with a no-return ds_add_u64 into ONE wave-private LDS histogram (integer adds: any lane may hit any bin).
//   LS   lane = segment, 20-bin rounds, exp2 recurrence (the production FX drain's access pattern)
//   G16  16-lane group = segment: one instruction covers 32 consecutive bins of the group's segment (16
//        consecutive u64 words: bank-conflict-free within the group), values by exp2 per bin
//   G8   8-lane group = segment, 16 bins per instruction
//   G16R as G16 with the exp2 recurrence at stride 32 (4 exp2 seeds per lane per segment)
//   LS*  LS on segments placed for distinct bank pairs: lane l's segments start on an even bin whose pair
//        index = l (mod 16) and their lengths are multiples of 20, so every 16-lane group of every
//        ds_add_u64 covers 16 distinct bank pairs (the bound for a conflict-free placement)
// Reports CU-cycles per 64 useful (in-segment) bin evaluations; the production float claim drain ran at
// ~13, the FX lane-serial drain at ~9.2 on C3.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

constexpr int kNR = 1024, kPadH = 1024 + 128;
constexpr int kSeg = 256;          // segments per wave
constexpr int kRep = 20;           // passes over a wave's segments
constexpr int kWG = 2048;          // workgroups (4 waves)
constexpr float kHL2E = 0.72134752044448170368f;
constexpr float kUnits = 20.0f;    // log2 of the fixed-point scale (values <= 1 -> <= 2^20 units)

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ unsigned cvt_rpi(float x) {
    int r;
    __asm__("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return (unsigned)r;
}
__device__ __forceinline__ void add2(unsigned long long* h, int pair, float v0, float v1) {
    const unsigned long long pv = ((unsigned long long)cvt_rpi(v1) << 32) | cvt_rpi(v0);
    __hip_atomic_fetch_add(h + pair, pv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

struct Seg { float ga, al, ks; int kl, len; };
static float hbits(int x) { float f; memcpy(&f, &x, 4); return f; }

// records float4 (ga, al + kUnits, t0 = kl - ks, kl | len << 16)
__device__ __forceinline__ void unpack(float4 r, int& kl, int& len) {
    kl = __float_as_int(r.w) & 0xFFFF;
    len = __float_as_int(r.w) >> 16;
}

template <int MODE>   // 0 LS, 1 G16, 2 G8, 3 G16R (MODE 0 also runs LS* on the placed records)
__global__ __launch_bounds__(256) void drain(const float4* __restrict__ recs, float* out) {
    __shared__ __align__(16) float4 rq[4][kSeg];
    __shared__ __align__(16) unsigned long long hist[4][kPadH / 2];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float4* src = recs + ((size_t)blockIdx.x * 4 + wave) * kSeg;
    for (int i = lane; i < kSeg; i += 64) rq[wave][i] = src[i];
    for (int i = lane; i < kPadH / 2; i += 64) hist[wave][i] = 0ull;
    __syncthreads();
    unsigned long long* h = hist[wave];
    for (int rep = 0; rep < kRep; ++rep) {
        if (MODE == 0) {
            // lane-serial: segments lane, lane + 64, ...; 20-bin rounds from the even bin at or below pos
            int idx = lane;
            float4 r = rq[wave][idx];
            int kl, len;
            unpack(r, kl, len);
            int pos = kl, rem = len;
            float t = r.z;
            while (__builtin_amdgcn_ballot_w64(idx < kSeg)) {
                if (idx < kSeg) {
                    const int o = pos & 1;
                    float cur = ex2(fmaf(r.x, t * t, r.y));
                    float q = ex2(r.x * fmaf(2.f, t, 1.f));
                    const float cc = ex2(2.f * r.x);
                    const int pb = pos >> 1;
#pragma unroll
                    for (int kv = 0; kv < 10; ++kv) {
                        const float v0 = (kv == 0 && o) ? 0.f : cur;
                        if (kv == 0) {
                            cur = o ? cur : cur * q;
                            q = o ? q : q * cc;
                        } else {
                            cur *= q;
                            q *= cc;
                        }
                        const float v1 = cur;
                        cur *= q;
                        q *= cc;
                        add2(h, pb + kv, v0, v1);
                    }
                    t += (float)(20 - o);
                    pos += 20 - o;
                    rem -= 20 - o;
                    if (rem <= 0) {
                        idx += 64;
                        r = rq[wave][min(idx, kSeg - 1)];
                        unpack(r, kl, len);
                        pos = kl; rem = len; t = r.z;
                    }
                }
            }
        } else {
            constexpr int GL = MODE == 2 ? 8 : 16;      // lanes per segment
            constexpr int NG = 64 / GL;
            const int grp = lane / GL, j = lane % GL;
            int idx = grp;
            float4 r = rq[wave][idx];
            int kl, len;
            unpack(r, kl, len);
            int p0 = kl >> 1, o = kl & 1, np = (len + o + 1) >> 1, c = 0;
            float ts = r.z - (float)o + 2.f * j;    // t of this lane's first bin in chunk 0
            float va = 0.f, vb = 0.f, ra = 0.f, rb = 0.f, C = 0.f;
            if (MODE == 3) {
                va = ex2(fmaf(r.x, ts * ts, r.y)); vb = ex2(fmaf(r.x, (ts + 1.f) * (ts + 1.f), r.y));
                const float S = 2.f * GL;   // bins per chunk
                ra = ex2(r.x * S * fmaf(2.f, ts, S)); rb = ex2(r.x * S * fmaf(2.f, ts + 1.f, S));
                C = ex2(2.f * S * S * r.x);
            }
            while (__builtin_amdgcn_ballot_w64(idx < kSeg)) {
                if (idx < kSeg) {
                    const int pr = c * GL + j;
                    if (pr < np) {
                        float v0, v1;
                        if (MODE == 3) {
                            v0 = va; v1 = vb;
                            va *= ra; ra *= C; vb *= rb; rb *= C;
                        } else {
                            const float t0 = ts + (float)(2 * GL * c), t1 = t0 + 1.f;
                            v0 = ex2(fmaf(r.x, t0 * t0, r.y));
                            v1 = ex2(fmaf(r.x, t1 * t1, r.y));
                        }
                        if (pr == 0 && o) v0 = 0.f;
                        add2(h, p0 + pr, v0, v1);
                    }
                    ++c;
                    if (c * GL >= np) {
                        idx += NG;
                        r = rq[wave][min(idx, kSeg - 1)];
                        unpack(r, kl, len);
                        p0 = kl >> 1; o = kl & 1; np = (len + o + 1) >> 1; c = 0;
                        ts = r.z - (float)o + 2.f * j;
                        if (MODE == 3) {
                            va = ex2(fmaf(r.x, ts * ts, r.y)); vb = ex2(fmaf(r.x, (ts + 1.f) * (ts + 1.f), r.y));
                            const float S = 2.f * GL;
                            ra = ex2(r.x * S * fmaf(2.f, ts, S)); rb = ex2(r.x * S * fmaf(2.f, ts + 1.f, S));
                            C = ex2(2.f * S * S * r.x);
                        }
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    unsigned s = 0;
    for (int i = lane; i < kPadH / 2; i += 64) s += (unsigned)(hist[wave][i] & 0xffff);
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}

static float timeit(void (*launch)(void*), void* arg) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch(arg);
    (void)hipDeviceSynchronize();
    hipEventRecord(a);
    launch(arg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = -1.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

struct Ctx { float* out; float4* recs; };

int main() {
    srand(7);
    auto urand = []() { return (rand() + 0.5) / ((double)RAND_MAX + 1.0); };
    const size_t nseg = (size_t)kWG * 4 * kSeg;
    std::vector<float4> recs(nseg), placed(nseg);
    double useful = 0, useful_p = 0;
    const float mc2 = 5.7f * 5.7f;
    for (size_t i = 0; i < nseg; ++i) {
        const double u = urand();
        const double g = exp(0.2 * sqrt(-2 * log(urand())) * cos(6.283185307 * urand()));
        int len = (int)(98.0 * g * sqrt(1 - u));
        len = std::max(1, std::min(len, 400));
        const int kl = (int)(urand() * (kNR - len - 40));
        const double hh = 0.5 * len + 0.5;
        const float ks = kl + 0.5f * (len - 1);
        const float ga = -kHL2E * mc2 * (float)(1 - u) / (float)(hh * hh);
        const float al = -kHL2E * mc2 * (float)u + kUnits;
        recs[i] = make_float4(ga, al, (float)kl - ks, hbits(kl | (len << 16)));
        useful += len;
        // placed copy: length rounded up to a multiple of 20, start pair = lane (mod 16)
        const int lanei = (int)(i % kSeg) % 64;
        const int lp = (len + 19) / 20 * 20;
        int kp = (int)(urand() * (kNR - lp - 40)) & ~31;
        kp += 2 * (lanei % 16);
        const double hp = 0.5 * lp + 0.5;
        const float ksp = kp + 0.5f * (lp - 1);
        const float gap = -kHL2E * mc2 * (float)(1 - u) / (float)(hp * hp);
        placed[i] = make_float4(gap, al, (float)kp - ksp, hbits(kp | (lp << 16)));
        useful_p += lp;
    }
    useful *= kRep;
    useful_p *= kRep;
    Ctx c;
    (void)hipMalloc(&c.out, (size_t)kWG * 256 * 4);
    (void)hipMalloc(&c.recs, nseg * sizeof(float4));
    (void)hipMemcpy(c.recs, recs.data(), nseg * sizeof(float4), hipMemcpyHostToDevice);
    const double cu_cyc = 2.4e9 * 256 * 1e-3;   // CU-cycles per ms
    float4* precs;
    (void)hipMalloc(&precs, nseg * sizeof(float4));
    (void)hipMemcpy(precs, placed.data(), nseg * sizeof(float4), hipMemcpyHostToDevice);
    const char* names[4] = {"LS  lane-serial 20-bin rounds", "G16 16 lanes/segment exp2/bin", "G8  8 lanes/segment exp2/bin",
                            "G16R 16 lanes/segment recurrence"};
    for (int m = 0; m < 4; ++m) {
        float ms;
        if (m == 0) ms = timeit([](void* a) { Ctx* c = (Ctx*)a; drain<0><<<kWG, 256>>>(c->recs, c->out); }, &c);
        else if (m == 1) ms = timeit([](void* a) { Ctx* c = (Ctx*)a; drain<1><<<kWG, 256>>>(c->recs, c->out); }, &c);
        else if (m == 2) ms = timeit([](void* a) { Ctx* c = (Ctx*)a; drain<2><<<kWG, 256>>>(c->recs, c->out); }, &c);
        else ms = timeit([](void* a) { Ctx* c = (Ctx*)a; drain<3><<<kWG, 256>>>(c->recs, c->out); }, &c);
        printf("%s: %.3f ms  %.2f CU-cycles per 64 useful\n", names[m], ms, ms * cu_cyc / (useful / 64));
    }
    Ctx cp = c;
    cp.recs = precs;
    const float ms = timeit([](void* a) { Ctx* c = (Ctx*)a; drain<0><<<kWG, 256>>>(c->recs, c->out); }, &cp);
    printf("LS* lane-serial, conflict-free placement: %.3f ms  %.2f CU-cycles per 64 useful\n", ms,
           ms * cu_cyc / (useful_p / 64));
    return 0;
}

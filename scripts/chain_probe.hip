// Latency probe for the single-wave selection kernel (k_sel): one wave per
// workgroup, 64 workgroups (as k_sel at cfg3), shader cycles (s_memtime) per
// repetition of each sequence, median over blocks.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/chain_probe scripts/chain_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define NREP 64

__device__ __forceinline__ unsigned long long now()
{
    unsigned long long t = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return t;
}
__device__ __forceinline__ void sync_v(double x)
{
    const int z = __builtin_amdgcn_readfirstlane((int)__double_as_longlong(x));
    asm volatile("s_nop 0" ::"s"(z));
}

template <int K>
__global__ void __launch_bounds__(64) probe(double *out, const double *in, unsigned long long *cyc, int n)
{
    if (blockIdx.x & 7u) return;
    const int lane = threadIdx.x;
    double a = in[lane], m = in[64 + lane], p = in[128 + lane];
    double r = 0.0;
    unsigned long long t0 = now();
    if constexpr (K == 0) {            // dependent v_fmac_f64, plain operands
        for (int i = 0; i < NREP; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a) : "v"(m), "v"(p));
        }
    } else if constexpr (K == 1) {     // dependent v_fmac_f64_dpp row_newbcast
        for (int i = 0; i < NREP; ++i) {
            asm volatile("s_nop 4\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                         : "+v"(a) : "v"(p), "v"(m));
        }
    } else if constexpr (K == 2) {     // two independent dependent chains interleaved (ILP 2), DPP
        double b = a + 1.0;
        for (int i = 0; i < NREP; ++i) {
            asm volatile("s_nop 4\n"
                         "v_fmac_f64_dpp %0, -%2, %3 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %1, -%2, %3 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%2, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %1, -%2, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%2, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %1, -%2, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %0, -%2, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                         "v_fmac_f64_dpp %1, -%2, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                         : "+v"(a), "+v"(b) : "v"(p), "v"(m));
        }
        a += b;
    } else if constexpr (K == 3) {     // dependent f64 division (IEEE, the compiler's sequence)
        for (int i = 0; i < NREP; ++i) {
#pragma unroll
            for (int u = 0; u < 2; ++u) a = a / p + 1.0;
        }
    } else if constexpr (K == 4) {     // wave minimum of a double (device.h wave_min form)
        for (int i = 0; i < NREP; ++i) {
            long long v = __double_as_longlong(a);
            auto step = [&](auto ctrl, int rm) {};
            (void)step;
#define DPPS(C, RM)                                                                                    \
    {                                                                                                  \
        const int lo = __builtin_amdgcn_update_dpp((int)v, (int)v, C, RM, 0xf, false);                 \
        const int hi = __builtin_amdgcn_update_dpp((int)(v >> 32), (int)(v >> 32), C, RM, 0xf, false); \
        const double o = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);                  \
        v = __double_as_longlong(fmin(__longlong_as_double(v), o));                                    \
    }
            DPPS(0xB1, 0xf) DPPS(0x4E, 0xf) DPPS(0x124, 0xf) DPPS(0x128, 0xf) DPPS(0x142, 0xa) DPPS(0x143, 0xc)
            const int lo = __builtin_amdgcn_readlane((int)v, 63);
            const int hi = __builtin_amdgcn_readlane((int)(v >> 32), 63);
            a = __longlong_as_double(((long long)hi << 32) | (unsigned)lo) + (double)(lane & 1);
        }
    } else if constexpr (K == 5) {     // wave minimum as two 32-bit unsigned passes on an order key
        for (int i = 0; i < NREP; ++i) {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(a);
            const unsigned long long key = (bits >> 63) ? ~bits : (bits | 0x8000000000000000ull);
            unsigned hk = (unsigned)(key >> 32);
#define UMIN(X, C, RM) X = min(X, (unsigned)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)X, C, RM, 0xf, false));
            UMIN(hk, 0xB1, 0xf) UMIN(hk, 0x4E, 0xf) UMIN(hk, 0x124, 0xf) UMIN(hk, 0x128, 0xf)
            UMIN(hk, 0x142, 0xa) UMIN(hk, 0x143, 0xc)
            const unsigned hmin = __builtin_amdgcn_readlane(hk, 63);
            unsigned lk = (unsigned)(key >> 32) == hmin ? (unsigned)key : 0xffffffffu;
            UMIN(lk, 0xB1, 0xf) UMIN(lk, 0x4E, 0xf) UMIN(lk, 0x124, 0xf) UMIN(lk, 0x128, 0xf)
            UMIN(lk, 0x142, 0xa) UMIN(lk, 0x143, 0xc)
            const unsigned lmin = __builtin_amdgcn_readlane(lk, 63);
            const unsigned long long kk = ((unsigned long long)hmin << 32) | lmin;
            const unsigned long long bb = (kk >> 63) ? (kk & 0x7fffffffffffffffull) : ~kk;
            a = __longlong_as_double((long long)bb) + (double)(lane & 1);
        }
    } else if constexpr (K == 6) {     // one 8-byte store + s_waitcnt vmcnt(0) (a drain), L2
        for (int i = 0; i < NREP; ++i) {
            __hip_atomic_store(out + 256 * blockIdx.x + lane, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            a += 1.0;
        }
    } else if constexpr (K == 7) {     // one sc1 (L1-bypass) 8-byte load, dependent (L2 hit)
        const double *q = out + 256 * blockIdx.x + lane;
        for (int i = 0; i < NREP; ++i) {
            a += __hip_atomic_load(q + (((long long)__double_as_longlong(a)) & 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if constexpr (K == 8) {     // readlane broadcast + plain f64 fma (8 values)
        for (int i = 0; i < NREP; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const double s = __longlong_as_double(
                    ((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(p) >> 32), u) << 32) |
                    (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(p), u));
                a = __builtin_fma(-s, m, a);
            }
        }
    } else if constexpr (K == 10) {    // dependent v_fmac_f64 with a scalar (SGPR) operand
        const long long pu = __builtin_amdgcn_readfirstlane((int)__double_as_longlong(p)) |
                             ((long long)__builtin_amdgcn_readfirstlane((int)(__double_as_longlong(p) >> 32)) << 32);
        for (int i = 0; i < NREP; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a) : "s"(pu), "v"(m));
        }
    } else if constexpr (K == 11) {    // dependent v_min_f64 (no DPP)
        for (int i = 0; i < NREP; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a) : "v"(m));
        }
    } else if constexpr (K == 12) {    // v_mov_b32_dpp quad_perm pair + v_min_f64 (one wmin step), x6
        for (int i = 0; i < NREP; ++i) {
            asm volatile("s_nop 1\n"
                         "v_mov_b32_dpp %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                         "v_mov_b32_dpp %2, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                         : "+v"(a), "=v"(r) : "v"(m), "v"(p));
        }
    } else if constexpr (K == 13) {    // wave minimum: order key, two u32 passes of single v_min_u32_dpp steps
        for (int i = 0; i < NREP; ++i) {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(a);
            const unsigned hi = (unsigned)(bits >> 32), lo = (unsigned)bits;
            const unsigned sg = (unsigned)((int)hi >> 31);
            unsigned hk = hi ^ (sg | 0x80000000u), lk = lo ^ sg;
#define UMIN1(X)                                                                                       \
    asm("s_nop 1\n"                                                                                   \
        "v_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"                  \
        "s_nop 1\n"                                                                                   \
        "v_min_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"                  \
        "s_nop 1\n"                                                                                   \
        "v_min_u32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n"                            \
        "s_nop 1\n"                                                                                   \
        "v_min_u32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n"                            \
        "s_nop 1\n"                                                                                   \
        "v_min_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"                         \
        "s_nop 1\n"                                                                                   \
        "v_min_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"                         \
        "s_nop 1\n"                                                                                   \
        : "+v"(X))
            unsigned hr = hk;
            UMIN1(hr);
            const unsigned hmin = __builtin_amdgcn_readlane(hr, 63);
            unsigned lr = hk == hmin ? lk : 0xffffffffu;
            UMIN1(lr);
            const unsigned lmin = __builtin_amdgcn_readlane(lr, 63);
            const unsigned s2 = (hmin >> 31) ? 0x80000000u : 0xffffffffu;
            const unsigned long long kk = ((unsigned long long)(hmin ^ s2) << 32) | (lmin ^ ((hmin >> 31) ? 0u : 0xffffffffu));
            a = __longlong_as_double((long long)kk) + (double)(lane & 1);
        }
    } else if constexpr (K == 9) {     // ballot + ctz + readlane (first lane with a property)
        for (int i = 0; i < NREP; ++i) {
            const unsigned long long bm = __ballot(a < p);
            const int f = bm ? __builtin_ctzll(bm) : 0;
            a += __longlong_as_double(
                ((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(m) >> 32), f) << 32) |
                (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(m), f));
        }
    }
    sync_v(a);
    const unsigned long long t1 = now();
    r = a;
    out[256 * blockIdx.x + 128 + lane] = r;
    if (lane == 0) cyc[blockIdx.x >> 3] = t1 - t0;
}

int main()
{
    const int G = 64;
    double *out, *in;
    unsigned long long *cyc;
    hipMalloc(&out, 256 * 8 * G * sizeof(double) * 8);
    hipMalloc(&in, 256 * sizeof(double));
    hipMalloc(&cyc, G * sizeof(unsigned long long));
    std::vector<double> h(256);
    for (int i = 0; i < 256; ++i) h[i] = 1.0 + 1e-3 * (i % 7);
    hipMemcpy(in, h.data(), 256 * 8, hipMemcpyHostToDevice);
    hipMemset(out, 0, 256 * 8 * G * sizeof(double) * 8);
    const char *names[] = {"fmac_f64 dep x8",  "fmac_f64_dpp dep x8", "fmac_f64_dpp 2 chains x4",
                           "div_f64 dep x2",    "wave_min f64 (dpp64)", "wave_min 2x u32 key",
                           "store+vmcnt(0)",    "load sc1 dep (L2)",   "readlane bcast+fma x8",
                           "ballot+ctz+readlane", "fmac_f64 sgpr dep x8", "v_min_f64 dep x8",
                           "2 dpp movs (issue)", "wave_min u32 dpp-min asm"};
    auto run = [&](auto kern, int k) {
        std::vector<unsigned long long> c(G);
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(kern, dim3(8 * G), dim3(64), 0, 0, out, in, cyc, 0);
            hipDeviceSynchronize();
        }
        hipMemcpy(c.data(), cyc, G * 8, hipMemcpyDeviceToHost);
        std::sort(c.begin(), c.end());
        printf("%-28s %7.1f cycles per repetition (median over %d blocks)\n", names[k], c[G / 2] / (double)NREP, G);
    };
    run(probe<0>, 0);
    run(probe<1>, 1);
    run(probe<2>, 2);
    run(probe<3>, 3);
    run(probe<4>, 4);
    run(probe<5>, 5);
    run(probe<6>, 6);
    run(probe<7>, 7);
    run(probe<8>, 8);
    run(probe<9>, 9);
    run(probe<10>, 10);
    run(probe<11>, 11);
    run(probe<13>, 13);
    return 0;
}

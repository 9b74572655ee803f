// f64 FMA issue-rate probe for the sweep's inner loop: the whole GPU runs
// waves of 8 independent accumulators, 256 FMAs each per repetition, with
// the multiplier operand
//   (a) broadcast by DPP (v_fmac_f64_dpp row_newbcast: k_sweep_dp's form),
//   (b) a scalar register (v_fma_f64 x, -s, p, x: a wave-uniform multiplier),
//   (c) a plain VGPR (v_fmac_f64),
// and reports f64 TFLOP/s (2 flops per FMA) against the 78.6 peak.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/fma_probe scripts/fma_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define REPS 256

template <int K>
__global__ void __launch_bounds__(256) fmak(double *out, const double *in, double s)
{
    const int lane = threadIdx.x;
    double x0 = in[lane], x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const double m = in[64 + (lane & 63)], p = in[128 + (lane & 63)];
    const double sv = __builtin_amdgcn_readfirstlane((int)__double_as_longlong(s)) == 0 ? s : s;
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (K == 0) {
                asm volatile("s_nop 1\n"
                             "v_fmac_f64_dpp %0, -%8, %9 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %1, -%8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %2, -%8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %3, -%8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %4, -%8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %5, -%8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %6, -%8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                             "v_fmac_f64_dpp %7, -%8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                             : "v"(m), "v"(p));
            } else if constexpr (K == 1) {
                asm volatile("v_fma_f64 %0, -%8, %9, %0\n"
                             "v_fma_f64 %1, -%8, %9, %1\n"
                             "v_fma_f64 %2, -%8, %9, %2\n"
                             "v_fma_f64 %3, -%8, %9, %3\n"
                             "v_fma_f64 %4, -%8, %9, %4\n"
                             "v_fma_f64 %5, -%8, %9, %5\n"
                             "v_fma_f64 %6, -%8, %9, %6\n"
                             "v_fma_f64 %7, -%8, %9, %7\n"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                             : "s"(sv), "v"(p));
            } else {
                asm volatile("v_fmac_f64 %0, %8, %9\n"
                             "v_fmac_f64 %1, %8, %9\n"
                             "v_fmac_f64 %2, %8, %9\n"
                             "v_fmac_f64 %3, %8, %9\n"
                             "v_fmac_f64 %4, %8, %9\n"
                             "v_fmac_f64 %5, %8, %9\n"
                             "v_fmac_f64 %6, %8, %9\n"
                             "v_fmac_f64 %7, %8, %9\n"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                             : "v"(m), "v"(p));
            }
        }
    }
    out[blockIdx.x * 256 + lane] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main()
{
    double *in, *out;
    hipMalloc(&in, 256 * sizeof(double));
    int nblk = 256 * 8;   // 8 blocks of 4 waves per CU: 8 waves per SIMD
    hipMalloc(&out, (size_t)nblk * 256 * sizeof(double));
    hipMemset(in, 0, 256 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"DPP broadcast (v_fmac_f64_dpp)", "scalar multiplier (v_fma_f64 s)", "plain (v_fmac_f64)"};
    auto run = [&](auto kern, int k) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), 0, 0, out, in, 0.5);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best) best = ms;
        }
        const double fmas = (double)nblk * 256 * REPS * 32;
        printf("%-34s %6.1f TFLOP/s f64 (%.3f ms)\n", names[k], 2 * fmas / (best * 1e-3) / 1e12, best);
    };
    for (int wps : {8, 4, 2, 1}) {
        nblk = 256 * wps;          // blocks of 4 waves: wps waves per SIMD
        printf("-- %d waves per SIMD\n", wps);
        run(fmak<0>, 0);
        run(fmak<1>, 1);
        run(fmak<2>, 2);
    }
    return 0;
}

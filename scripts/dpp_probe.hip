// VALU probe (diagnostic, not product code): issue rate of v_fmac_f64 with a
// DPP row_newbcast operand (the k_sweep_dp inner loop) against the plain
// v_fmac_f64, 8 independent accumulators per lane, 4 waves per SIMD on every
// CU.  Prints FMA/s per variant.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/dpp_probe scripts/dpp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                          \
        }                                                                      \
    } while (0)

#define F8(OP, SUF)                                                                                 \
    OP " %0, -%8, %9" SUF "\n" OP " %1, -%8, %9" SUF "\n" OP " %2, -%8, %9" SUF "\n" OP " %3, -%8, %9" SUF \
       "\n" OP " %4, -%8, %9" SUF "\n" OP " %5, -%8, %9" SUF "\n" OP " %6, -%8, %9" SUF "\n" OP          \
       " %7, -%8, %9" SUF "\n"

#define G1(A) "v_fma_f64 " A ", -%8, %9, " A "\n"
#define G8 G1("%0") G1("%1") G1("%2") G1("%3") G1("%4") G1("%5") G1("%6") G1("%7")

template <int DPP>
__global__ void __launch_bounds__(256) k_fma(double *out, int iters, double m, double p)
{
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    double mv = m * threadIdx.x, pv = p;
    for (int i = 0; i < iters; ++i) {
        if (DPP)
            asm volatile("s_nop 1\n" F8("v_fmac_f64_dpp", " row_newbcast:5 row_mask:0xf bank_mask:0xf")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(mv), "v"(pv));
        else
            asm volatile("s_nop 1\n" G8
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(mv), "v"(pv));
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 4, iters = 20000;   // 4 workgroups of 4 waves per CU: 4 waves per SIMD
    double *out = nullptr;
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int dpp = 0; dpp < 2; ++dpp)
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            if (dpp)
                hipLaunchKernelGGL(k_fma<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-9, 0.5);
            else
                hipLaunchKernelGGL(k_fma<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-9, 0.5);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double fmas = (double)blocks * 256 * iters * 8;
            std::printf("{\"variant\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"TFMA_per_s\": %.2f}\n",
                        dpp ? "v_fmac_f64_dpp row_newbcast" : "v_fmac_f64", rep, ms, fmas / (ms * 1e-3) / 1e12);
        }
    return 0;
}

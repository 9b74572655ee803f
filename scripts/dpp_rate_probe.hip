// f64 FMA rate of the sweep's inner-loop form at the sweep's occupancy:
// 8 accumulators, the multiplier broadcast by DPP (v_fmac_f64_dpp
// row_newbcast, k_sweep_rl's rg_pair) against plain v_fmac_f64, at two waves
// per SIMD (64 KB of LDS per 4-wave block: 2 blocks per CU) and at eight.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/dpp_rate_probe scripts/dpp_rate_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define REPS 1024
#define RGF(XK, P, L) "v_fmac_f64_dpp %" #XK ", -%8, %" #P " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
#define PF(XK, P) "v_fmac_f64 %" #XK ", -%8, %" #P "\n"

template <bool DPP>
__global__ void __launch_bounds__(256) rate(double *out, const double *in)
{
    extern __shared__ double pad[];
    const int l = threadIdx.x;
    double x[8];
    for (int k = 0; k < 8; ++k) x[k] = in[l & 63] + k;
    double m = in[64 + (l & 63)], pa = in[128 + (l & 63)], pb = in[192 + (l & 63)];
    for (int r = 0; r < REPS; ++r) {
        if constexpr (DPP)
            asm volatile("s_nop 1\n" RGF(0, 9, 0) RGF(1, 9, 1) RGF(2, 9, 2) RGF(3, 9, 3) RGF(4, 9, 4) RGF(5, 9, 5)
                             RGF(6, 9, 6) RGF(7, 9, 7) RGF(0, 10, 8) RGF(1, 10, 9) RGF(2, 10, 10) RGF(3, 10, 11)
                                 RGF(4, 10, 12) RGF(5, 10, 13) RGF(6, 10, 14) RGF(7, 10, 15)
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7])
                         : "v"(m), "v"(pa), "v"(pb));
        else
            asm volatile(PF(0, 9) PF(1, 9) PF(2, 9) PF(3, 9) PF(4, 9) PF(5, 9) PF(6, 9) PF(7, 9) PF(0, 10) PF(1, 10)
                             PF(2, 10) PF(3, 10) PF(4, 10) PF(5, 10) PF(6, 10) PF(7, 10)
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7])
                         : "v"(m), "v"(pa), "v"(pb));
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    if (l == 0) pad[0] = s;
    out[blockIdx.x * 256 + l] = s;
}

int main()
{
    double *out, *in;
    hipMalloc(&out, 4096 * 256 * 8);
    hipMalloc(&in, 256 * 8);
    hipMemset(in, 0, 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int dpp = 0; dpp < 2; ++dpp)
        for (int occ = 0; occ < 2; ++occ) {
            const int blocks = occ ? 2048 : 512;          // 8 or 2 waves per SIMD
            const size_t lds = occ ? 0 : 64 * 1024;
            auto k = dpp ? rate<true> : rate<false>;
            for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, out, in);
            hipEventRecord(e0);
            for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, out, in);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double fmas = 5.0 * blocks * 256.0 * REPS * 16;
            printf("{\"probe\": \"f64 fma rate\", \"form\": \"%s\", \"waves_per_simd\": %d, \"TFMA_s\": %.2f}\n",
                   dpp ? "v_fmac_f64_dpp row_newbcast (rg_pair)" : "v_fmac_f64", occ ? 8 : 2,
                   fmas / (ms * 1e-3) / 1e12);
        }
    return 0;
}

// HBM ceilings at cfg4's size (diagnostic, not product code): a
// 32769 x 8320 float64 buffer (2.18 GB, far beyond the 256 MB Infinity
// Cache), updated in place with 16-byte accesses:
//   linear   : grid-stride in-place pass (4 workgroups of 256 per CU)
//   strip    : the sweep's pattern -- a workgroup of 8 waves owns a 128-column
//              strip of a run of rows, each wave 4-row batches (2 workgroups
//              per CU, as k_sweep_dp at 64 pivots), with NF dependent FMAs per
//              element per pass (0: a plain scale)
// Prints us and GB/s (median of 11 launches) per pattern.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/cfg4_probe scripts/cfg4_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__global__ void k_inplace(double2 *a, long long n2, double s)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n2;
         i += (long long)gridDim.x * blockDim.x) {
        double2 v = a[i];
        v.x *= s;
        v.y *= s;
        a[i] = v;
    }
}

template <int NF>
__global__ void __launch_bounds__(512) k_strip(double *T, long long ld, long long rows, int nstrips,
                                               long long run, double s)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int strip = blockIdx.x % nstrips;
    const long long r0 = (long long)(blockIdx.x / nstrips) * run, r1 = min(rows, r0 + run);
    const long long c = (long long)strip * 128 + lane * 2;
    if (c + 1 >= ld) return;
    for (long long rb = r0 + wave * 4; rb < r1; rb += 32) {
        double2 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = *reinterpret_cast<double2 *>(T + min(rb + k, r1 - 1) * ld + c);
#pragma unroll 8
        for (int f = 0; f < (NF > 0 ? NF : 1); ++f)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[k].x = NF > 0 ? fma(-s, 1e-300, x[k].x) : x[k].x * s;
                x[k].y = NF > 0 ? fma(-s, 1e-300, x[k].y) : x[k].y * s;
            }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (rb + k < r1) *reinterpret_cast<double2 *>(T + (rb + k) * ld + c) = x[k];
    }
}

int main()
{
    const long long rows = 32769, ld = 8320, n = rows * ld;
    double *a = nullptr;
    CK(hipMalloc(&a, n * 8));
    CK(hipMemset(a, 0, n * 8));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        std::vector<float> ms;
        for (int it = 0; it < 14; ++it) {
            (void)hipEventRecord(e0, 0);
            launch();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float t = 0.f;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (it >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        return ms[ms.size() / 2] * 1e-3;
    };
    const double bytes = 2.0 * n * 8;
    for (int wg : {4, 8}) {
        const double t = timeit([&] { hipLaunchKernelGGL(k_inplace, dim3(ncu * wg), dim3(256), 0, 0, (double2 *)a, n / 2, 1.0); });
        std::printf("{\"pattern\": \"linear-inplace\", \"workgroups_per_cu\": %d, \"us\": %.1f, \"GBps\": %.0f}\n", wg,
                    t * 1e6, bytes / t / 1e9);
        std::fflush(stdout);
    }
    const int ns = (int)((ld + 127) / 128);
    for (int bpc : {2, 3}) {
        long long nrun = (long long)ncu * bpc / ns;
        long long run = (rows + nrun - 1) / nrun;
        run = (run + 3) / 4 * 4;
        nrun = (rows + run - 1) / run;
        for (int nf : {0, 32, 64}) {
            const double t = timeit([&] {
                if (nf == 0) hipLaunchKernelGGL(k_strip<0>, dim3(nrun * ns), dim3(512), 0, 0, a, ld, rows, ns, run, 1.0);
                else if (nf == 32) hipLaunchKernelGGL(k_strip<32>, dim3(nrun * ns), dim3(512), 0, 0, a, ld, rows, ns, run, 1.0);
                else hipLaunchKernelGGL(k_strip<64>, dim3(nrun * ns), dim3(512), 0, 0, a, ld, rows, ns, run, 1.0);
            });
            std::printf("{\"pattern\": \"strip-inplace\", \"fma_per_element\": %d, \"workgroups_per_cu\": %d, \"us\": %.1f, \"GBps\": %.0f}\n",
                        nf, bpc, t * 1e6, bytes / t / 1e9);
            std::fflush(stdout);
        }
    }
    return 0;
}

// HBM ceilings for the sweep's access pattern (diagnostic, not product code):
// a 270.6 MB float64 buffer (cfg3's tableau) streamed with 16-byte accesses
//   read   : sum every element (one read)
//   copy   : B <- A (read + write to another buffer)
//   inplace: A <- A * s (read + write of the same lines: the sweep's pattern)
// Prints GB/s per pattern (median of 20 launches, HIP events).
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

__global__ void k_read(const double2 *a, long long n2, double *out)
{
    double2 acc = make_double2(0.0, 0.0);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n2;
         i += (long long)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        acc.x += v.x;
        acc.y += v.y;
    }
    if (acc.x == 12345.678) out[0] = acc.y;   // keeps the loads
}

__global__ void k_copy(const double2 *a, double2 *b, long long n2)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n2;
         i += (long long)gridDim.x * blockDim.x)
        b[i] = a[i];
}

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

// the sweep's pattern: workgroup = 8 waves on a 128-column strip of a run of
// rows, each wave 4 rows (16 B per lane per row) per batch, NF dependent FMAs
// per element per pass (0: plain scale)
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
#pragma unroll
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

// the same, runs interleaved: workgroup j of a strip takes the 32-row batches
// j, j + nrun, j + 2 nrun, ... so every workgroup works inside one moving
// window of nrun x 32 rows
template <int NF>
__global__ void __launch_bounds__(512) k_strip_il(double *T, long long ld, long long rows, int nstrips,
                                                  int nrun, double s)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int strip = blockIdx.x % nstrips;
    const int j = blockIdx.x / nstrips;
    const long long c = (long long)strip * 128 + lane * 2;
    if (c + 1 >= ld) return;
    for (long long bb = j; bb * 32 < rows; bb += nrun) {
        const long long rb = bb * 32 + wave * 4;
        if (rb >= rows) continue;
        double2 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = *reinterpret_cast<double2 *>(T + min(rb + k, rows - 1) * ld + c);
#pragma unroll
        for (int f = 0; f < (NF > 0 ? NF : 1); ++f)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[k].x = NF > 0 ? fma(-s, 1e-300, x[k].x) : x[k].x * s;
                x[k].y = NF > 0 ? fma(-s, 1e-300, x[k].y) : x[k].y * s;
            }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (rb + k < rows) *reinterpret_cast<double2 *>(T + (rb + k) * ld + c) = x[k];
    }
}

// strips of 256 columns: each lane 32 contiguous bytes per row (two 16-byte
// accesses), so one wave-instruction pair covers 2 KB of a row
template <int NF>
__global__ void __launch_bounds__(512) k_strip256(double *T, long long ld, long long rows, int nstrips,
                                                  long long run, double s)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int strip = blockIdx.x % nstrips;
    const long long r0 = (long long)(blockIdx.x / nstrips) * run, r1 = min(rows, r0 + run);
    const long long c = (long long)strip * 256 + lane * 4;
    if (c + 3 >= ld) return;
    for (long long rb = r0 + wave * 4; rb < r1; rb += 32) {
        double2 x[4][2];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                x[k][h] = *reinterpret_cast<double2 *>(T + min(rb + k, r1 - 1) * ld + c + 2 * h);
#pragma unroll
        for (int f = 0; f < (NF > 0 ? NF : 1); ++f)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    x[k][h].x = NF > 0 ? fma(-s, 1e-300, x[k][h].x) : x[k][h].x * s;
                    x[k][h].y = NF > 0 ? fma(-s, 1e-300, x[k][h].y) : x[k][h].y * s;
                }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (rb + k < r1)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    *reinterpret_cast<double2 *>(T + (rb + k) * ld + c + 2 * h) = x[k][h];
    }
}

int main()
{
    const long long n = 4097LL * 8256LL;     // cfg3: (m + 1) x ld doubles
    const long long n2 = n / 2;
    double2 *a = nullptr, *b = nullptr;
    double *o = nullptr;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    CK(hipMalloc(&o, 8));
    CK(hipMemset(a, 0, n * 8));
    CK(hipMemset(b, 0, n * 8));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int wg : {4, 8}) {
        const dim3 grid(ncu * wg), blk(256);
        for (int p = 0; p < 3; ++p) {
            std::vector<float> ms;
            for (int it = 0; it < 23; ++it) {
                CK(hipEventRecord(e0, 0));
                if (p == 0) hipLaunchKernelGGL(k_read, grid, blk, 0, 0, a, n2, o);
                else if (p == 1) hipLaunchKernelGGL(k_copy, grid, blk, 0, 0, a, b, n2);
                else hipLaunchKernelGGL(k_inplace, grid, blk, 0, 0, a, n2, 1.0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0.f;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (it >= 3) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2] * 1e-3;
            const double bytes = (p == 0 ? 1.0 : 2.0) * n * 8;
            std::printf("{\"pattern\": \"%s\", \"workgroups_per_cu\": %d, \"bytes\": %.0f, \"us\": %.1f, \"GBps\": %.0f}\n",
                        p == 0 ? "read" : p == 1 ? "copy" : "inplace", wg, bytes, med * 1e6,
                        bytes / med / 1e9);
        }
    }
    // strip pattern at cfg3's shape: 4097 rows x 8256, 65 strips, 11 runs (3 workgroups per CU)
    {
        const long long ld = 8256, rows = 4097;
        const int ns = (int)((ld + 127) / 128);
        for (int bpc : {3, 4}) {
            long long nrun = (long long)ncu * bpc / ns;
            long long run = (rows + nrun - 1) / nrun;
            run = (run + 3) / 4 * 4;
            nrun = (rows + run - 1) / run;
            for (int nf : {0, 32}) {
                std::vector<float> ms;
                for (int it = 0; it < 23; ++it) {
                    CK(hipEventRecord(e0, 0));
                    if (nf == 0) hipLaunchKernelGGL(k_strip<0>, dim3(nrun * ns), dim3(512), 0, 0, (double *)a, ld, rows, ns, run, 1.0);
                    else hipLaunchKernelGGL(k_strip<32>, dim3(nrun * ns), dim3(512), 0, 0, (double *)a, ld, rows, ns, run, 1.0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float t = 0.f;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    if (it >= 3) ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2] * 1e-3;
                const double bytes = 2.0 * n * 8;
                std::printf("{\"pattern\": \"strip-inplace\", \"fma_per_element\": %d, \"workgroups_per_cu\": %d, \"us\": %.1f, \"GBps\": %.0f}\n",
                            nf, bpc, med * 1e6, bytes / med / 1e9);
            }
        }
    }
    // 256-column strips (2 KB of a row per wave)
    {
        const long long ld = 8256, rows = 4097;
        const int ns = (int)((ld + 255) / 256);
        for (int bpc : {2, 3}) {
            long long nrun = (long long)ncu * bpc / ns;
            long long run = (rows + nrun - 1) / nrun;
            run = (run + 3) / 4 * 4;
            nrun = (rows + run - 1) / run;
            for (int nf : {0, 32}) {
                std::vector<float> ms;
                for (int it = 0; it < 23; ++it) {
                    CK(hipEventRecord(e0, 0));
                    if (nf == 0) hipLaunchKernelGGL(k_strip256<0>, dim3(nrun * ns), dim3(512), 0, 0, (double *)a, ld, rows, ns, run, 1.0);
                    else hipLaunchKernelGGL(k_strip256<32>, dim3(nrun * ns), dim3(512), 0, 0, (double *)a, ld, rows, ns, run, 1.0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float t = 0.f;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    if (it >= 3) ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2] * 1e-3;
                std::printf("{\"pattern\": \"strip256-inplace\", \"fma_per_element\": %d, \"workgroups_per_cu\": %d, \"us\": %.1f, \"GBps\": %.0f}\n",
                            nf, bpc, med * 1e6, 2.0 * n * 8 / med / 1e9);
            }
        }
    }
    // strip pattern, runs interleaved into one moving window
    {
        const long long ld = 8256, rows = 4097;
        const int ns = (int)((ld + 127) / 128);
        const int nrun = ncu * 3 / ns;
        for (int nf : {0, 32}) {
            std::vector<float> ms;
            for (int it = 0; it < 23; ++it) {
                CK(hipEventRecord(e0, 0));
                if (nf == 0) hipLaunchKernelGGL(k_strip_il<0>, dim3(nrun * ns), dim3(512), 0, 0, (double *)a, ld, rows, ns, nrun, 1.0);
                else hipLaunchKernelGGL(k_strip_il<32>, dim3(nrun * ns), dim3(512), 0, 0, (double *)a, ld, rows, ns, nrun, 1.0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0.f;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (it >= 3) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2] * 1e-3;
            std::printf("{\"pattern\": \"strip-inplace-interleaved\", \"fma_per_element\": %d, \"us\": %.1f, \"GBps\": %.0f}\n",
                        nf, med * 1e6, 2.0 * n * 8 / med / 1e9);
        }
    }
    // the same in-place pass over a 2x larger buffer (does not fit the 256 MB Infinity Cache)
    {
        double2 *c = nullptr;
        const long long nn = 2 * n;
        CK(hipMalloc(&c, nn * 8));
        CK(hipMemset(c, 0, nn * 8));
        std::vector<float> ms;
        for (int it = 0; it < 13; ++it) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_inplace, dim3(ncu * 4), dim3(256), 0, 0, c, nn / 2, 1.0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t = 0.f;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2] * 1e-3;
        std::printf("{\"pattern\": \"inplace-541MB\", \"us\": %.1f, \"GBps\": %.0f}\n", med * 1e6, 2.0 * nn * 8 / med / 1e9);
    }
    return 0;
}

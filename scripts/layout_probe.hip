// Tableau layout probe (diagnostic, not product code): what the selection's
// two gathers cost per pivot under tiled storage.  k_sel's blocks (64 single
// waves on ONE XCD: grid 512, blocks 0, 8, 16, ... work) load
//   column gather: element (r, C) of each own row (lane l: row 1 + 64 b + l),
//   row gather:    elements (R, j) of the block's 128 own columns (2 per lane),
// with the tableau stored in tiles of A rows x B columns (A x B x 8 bytes
// contiguous, tiles row-major over the tile grid; A = 1 is today's row-major
// layout with pitch ld).  Per layout: the mean and the slowest block's time of
// each gather (100 MHz clock, median over iterations), warm (the tableau read
// repeatedly: Infinity-Cache hits where it fits) and after streaming a 1 GiB
// scratch buffer (cold).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/layout_probe scripts/layout_probe.hip
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

struct Lay {
    int A, B;           // tile rows, tile columns
    long long tpr;      // tiles per tile-row
};
__device__ __forceinline__ long long at(const Lay &L, long long r, long long c)
{
    const long long tr = r / L.A, tc = c / L.B;
    return ((tr * L.tpr + tc) * L.A + (r % L.A)) * L.B + (c % L.B);
}

__global__ void __launch_bounds__(64) k_col(const double *T, Lay L, long long rows, long long C, long long *stamp,
                                            double *sink)
{
    if (blockIdx.x & 7u) return;
    const unsigned b = blockIdx.x >> 3;
    const long long r = 1 + 64LL * b + threadIdx.x;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    const double a = r < rows ? T[at(L, r, C)] : 0.0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = (long long)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        stamp[2 * b] = t0;
        stamp[2 * b + 1] = t1;
    }
    if (a == 1234.5) sink[0] = a;
}
__global__ void __launch_bounds__(64) k_row(const double *T, Lay L, long long cols, long long R, long long *stamp,
                                            double *sink)
{
    if (blockIdx.x & 7u) return;
    const unsigned b = blockIdx.x >> 3;
    const long long c0 = 1 + 128LL * b + threadIdx.x, c1 = c0 + 64;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    const double x0 = c0 < cols ? T[at(L, R, c0)] : 0.0;
    const double x1 = c1 < cols ? T[at(L, R, c1)] : 0.0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = (long long)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        stamp[2 * b] = t0;
        stamp[2 * b + 1] = t1;
    }
    if (x0 + x1 == 1234.5) sink[0] = x0;
}
__global__ void k_stream(double *S, long long n, double *sink)
{
    double s = 0.0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        s += S[i];
    if (s == 1234.5) sink[0] = s;
}

int main()
{
    const long long rows = 4097, cols = 8193, ld = 8320;
    const long long scratch_n = (1LL << 30) / 8;
    double *T = nullptr, *S = nullptr, *sink = nullptr;
    long long *st = nullptr;
    const long long cap = (rows + 16) * (ld + 16);
    CK(hipMalloc(&T, cap * sizeof(double)));
    CK(hipMemset(T, 0, cap * sizeof(double)));
    CK(hipMalloc(&S, scratch_n * sizeof(double)));
    CK(hipMemset(S, 0, scratch_n * sizeof(double)));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&st, 2 * 64 * sizeof(long long)));
    std::vector<long long> h(2 * 64);
    const int lays[][2] = {{1, 8320}, {2, 8}, {2, 16}, {4, 4}, {4, 8}, {4, 16}, {8, 8}, {8, 16}, {16, 8}, {16, 16}};
    for (auto &l : lays) {
        Lay L{l[0], l[1], (ld + l[1] - 1) / l[1]};
        if ((long long)((rows + L.A - 1) / L.A) * L.tpr * L.A * L.B > cap) return 2;
        for (int cold = 0; cold < 2; ++cold) {
            std::vector<double> cm, cx, rm, rx;
            for (int it = 0; it < 40; ++it) {
                const long long C = 1 + (it * 2654435761LL) % 8192, R = 1 + (it * 40503LL) % 4096;
                for (int g = 0; g < 2; ++g) {
                    if (cold) hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, 0, S, scratch_n, sink);
                    if (g == 0)
                        hipLaunchKernelGGL(k_col, dim3(512), dim3(64), 0, 0, T, L, rows, C, st, sink);
                    else
                        hipLaunchKernelGGL(k_row, dim3(512), dim3(64), 0, 0, T, L, cols, R, st, sink);
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(h.data(), st, 2 * 64 * sizeof(long long), hipMemcpyDeviceToHost));
                    if (it < 5) continue;
                    double sum = 0.0, mx = 0.0;
                    for (int b = 0; b < 64; ++b) {
                        const double d = (h[2 * b + 1] - h[2 * b]) * 0.01;
                        sum += d;
                        mx = std::max(mx, d);
                    }
                    (g == 0 ? cm : rm).push_back(sum / 64);
                    (g == 0 ? cx : rx).push_back(mx);
                }
            }
            auto med = [](std::vector<double> v) {
                std::sort(v.begin(), v.end());
                return v[v.size() / 2];
            };
            std::printf("{\"tile\": \"%dx%d\", \"cold\": %d, \"col_mean_us\": %.3f, \"col_max_us\": %.3f, "
                        "\"row_mean_us\": %.3f, \"row_max_us\": %.3f}\n",
                        L.A, L.B == 8320 ? 0 : L.B, cold, med(cm), med(cx), med(rm), med(rx));
            std::fflush(stdout);
        }
    }
    return 0;
}

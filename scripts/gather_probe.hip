// Column-gather probe (diagnostic, not product code): the selection's
// "column C of every own row" load, one 8-byte element per tableau row, as
// k_group issues it (G single-wave blocks, RPL rows per lane, all loads in
// flight before the first wait), over a float64 buffer with row pitch
// ld doubles.  Each block stamps the 100 MHz clock before its loads and after
// they have all returned; per launch: the span from the first block's start
// to the last block's end, and the mean per-block time.  Prints one JSON
// line per (rows, pitch).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/gather_probe scripts/gather_probe.hip
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

template <int RPL>
__global__ void __launch_bounds__(64) k_gather(const double *T, long long ld, long long rows, long long C,
                                               long long rpb, long long *stamp, double *sink)
{
    const long long r0 = 1 + blockIdx.x * rpb;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    double a[RPL];
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        const long long i = r0 + threadIdx.x + 64 * k;
        a[k] = (i < rows && i < r0 + rpb) ? T[i * ld + C] : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < RPL; ++k) s += a[k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = (long long)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        stamp[2 * blockIdx.x] = t0;
        stamp[2 * blockIdx.x + 1] = t1;
    }
    if (s == 1234.5) sink[0] = s;
}

int main()
{
    const long long maxrows = 32769, maxld = 64LL * 272;   // every pitch below fits
    double *T = nullptr, *sink = nullptr;
    long long *st = nullptr;
    CK(hipMalloc(&T, maxrows * maxld * sizeof(double)));
    CK(hipMemset(T, 0, maxrows * maxld * sizeof(double)));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&st, 2 * 512 * sizeof(long long)));
    std::vector<long long> h(2 * 512);
    // pitch in units of 64 doubles (512 B): 129 is the engine's cfg3/cfg4 pitch
    std::vector<int> pitches;
    for (int p = 8; p <= 272; ++p) pitches.push_back(p);
    for (long long rows : {32769LL, 4097LL}) {
        const int G = rows > 5000 ? 256 : 64;
        const long long rpb = (rows - 1 + G - 1) / G;
        for (int p : pitches) {
            const long long ld = 64LL * p;
            if (ld > maxld) return 2;   // never past the buffer
            std::vector<double> span, mean, maxb;
            for (int it = 0; it < 30; ++it) {
                const long long C = 1 + (it * 2654435761LL) % std::min(8192LL, ld - 1);
                if (rpb > 64)
                    hipLaunchKernelGGL(k_gather<2>, dim3(G), dim3(64), 0, 0, T, ld, rows, C, rpb, st, sink);
                else
                    hipLaunchKernelGGL(k_gather<1>, dim3(G), dim3(64), 0, 0, T, ld, rows, C, rpb, st, sink);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h.data(), st, 2 * G * sizeof(long long), hipMemcpyDeviceToHost));
                if (it < 6) continue;   // warm-up
                long long s0 = h[0], s1 = h[1];
                double sum = 0.0, mx = 0.0;
                for (int b = 0; b < G; ++b) {
                    s0 = std::min(s0, h[2 * b]);
                    s1 = std::max(s1, h[2 * b + 1]);
                    const double d = (h[2 * b + 1] - h[2 * b]) * 0.01;
                    sum += d;
                    mx = std::max(mx, d);
                }
                span.push_back((s1 - s0) * 0.01);
                mean.push_back(sum / G);
                maxb.push_back(mx);
            }
            auto med = [](std::vector<double> v) {
                std::sort(v.begin(), v.end());
                return v[v.size() / 2];
            };
            std::printf("{\"rows\": %lld, \"blocks\": %d, \"pitch_bytes\": %lld, \"span_us\": %.2f, "
                        "\"block_mean_us\": %.2f, \"block_max_us\": %.2f}\n",
                        rows, G, ld * 8, med(span), med(mean), med(maxb));
            std::fflush(stdout);
        }
    }
    return 0;
}

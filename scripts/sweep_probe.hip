// Where the cfg4 sweep's time goes (diagnostic, not product code): the
// product's k_sweep_dp structure (128-column strips, 8 waves x 4-row batches,
// next batch in flight, P slice in LDS, DPP-broadcast multipliers) on a
// cfg4-sized buffer (32769 x 8320 float64, 64 pivots), with parts switched off
// by MODE bits -- results are not checked, only times:
//   1  no multiplier loads (constant multiplier registers)
//   2  no P reads from LDS in the loop (constant P registers)
//   4  plain FMAs (the lane's own multiplier) instead of the DPP operand
//   8  no FMAs
//  16  no write-through (sc1) on the stores
//  32  multipliers loaded by one 16-lane row only (the others idle)
//  64  multipliers as 16-byte loads, 8 a batch instead of 16 8-byte ones
// 128  XCD-grouped tiles: each XCD takes a contiguous range of (run, strip) tiles
// 256  tableau loads non-temporal (aux nt); 512 tableau loads sc0
// 1024 multipliers batch-interleaved: a 4-row batch's 4-pivot chunk is one 128-byte line
// Prints us and GB/s (median of 9 launches) per mode.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/sweep_probe scripts/sweep_probe.hip
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

typedef unsigned v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}

#define DPF(XR, PV, L) "v_fmac_f64_dpp " XR ", -%8, " PV " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
#define DPP_PIVOT(L0, L1, L2, L3, PX, PY)                                                     \
    DPF("%0", PX, L0) DPF("%1", PY, L0) DPF("%2", PX, L1) DPF("%3", PY, L1) DPF("%4", PX, L2) \
    DPF("%5", PY, L2) DPF("%6", PX, L3) DPF("%7", PY, L3)
#define DPP_OUTS(x)                                                                                       \
    "+v"(x[0].x), "+v"(x[0].y), "+v"(x[1].x), "+v"(x[1].y), "+v"(x[2].x), "+v"(x[2].y), "+v"(x[3].x), \
        "+v"(x[3].y)
template <int MODE>
__device__ __forceinline__ void dp_half(double2 (&x)[4], double m, double2 p0, double2 p1, int h)
{
    if (MODE & 8) return;
    if (MODE & 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[k].x = fma(-m, p0.x, x[k].x);
            x[k].y = fma(-m, p0.y, x[k].y);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[k].x = fma(-m, p1.x, x[k].x);
            x[k].y = fma(-m, p1.y, x[k].y);
        }
        return;
    }
    if (h == 0)
        asm("s_nop 1\n" DPP_PIVOT(0, 1, 2, 3, "%9", "%10") DPP_PIVOT(4, 5, 6, 7, "%11", "%12")
            : DPP_OUTS(x) : "v"(m), "v"(p0.x), "v"(p0.y), "v"(p1.x), "v"(p1.y));
    else
        asm(DPP_PIVOT(8, 9, 10, 11, "%9", "%10") DPP_PIVOT(12, 13, 14, 15, "%11", "%12")
            : DPP_OUTS(x) : "v"(m), "v"(p0.x), "v"(p0.y), "v"(p1.x), "v"(p1.y));
}

template <int MODE>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_probe(double *T, const double *__restrict__ P, const double *__restrict__ M, long long ld, long long rows,
        int nstrips, long long run, int nd, int ntiles)
{
    constexpr int W = 8, NB = 64, RW = 4, NM = NB / 4;
    constexpr int SA = (MODE & 16) ? 0 : 16;
    __shared__ double2 sp[NB][64];
    unsigned bid = blockIdx.x;
    if (MODE & 128) {         // XCD-grouped: XCD x (blocks x, x + 8, ...) takes a contiguous range of (run, strip) tiles
        const unsigned per = gridDim.x / 8;
        bid = (bid % 8) * per + bid / 8;
        if (bid >= (unsigned)ntiles) return;
    }
    const int strip = (int)(bid % (unsigned)nstrips);
    const long long r0 = (long long)(bid / (unsigned)nstrips) * run;
    const long long r1 = min(rows, r0 + run);
    if (r0 >= r1) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long c0 = (long long)strip * 128;
    const int lo = min(lane * 2, (int)(ld - c0) - 2);
    const int lob = lo * 8, ldb = (int)(ld * 8);
    const double *Ts = T + c0;
    double *Tos = T + c0;
    for (int s = wave; s < NB; s += W) sp[s][lane] = *reinterpret_cast<const double2 *>(P + s * ld + c0 + lo);
    const int q = lane & 15, qs = q >> 2, qk = q & 3;
    const int nch = (nd + 3) >> 2;
    auto load_m = [&](long long rb, int c) {
        if (MODE & 1) return 1e-3;
        if (MODE & 32) {      // one 16-lane row loads (no 4x replication of the addresses)
            if (lane >= 16) return 0.0;
        }
        if (MODE & 64) {      // b128 pairs: chunk c's odd half comes with the even one (8 loads a batch)
            if (c & 1) return 0.0;
            const int mk2 = min(qk & 2, (int)(r1 - 1 - rb));
            const int sv2 = min(4 * c + (q >> 1), nd - 1);
            const double2 v = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(M + rb), (sv2 * (int)rows + mk2) * 8, 0, 0));
            return v.x + v.y;
        }
        if (MODE & 1024) {    // batch-interleaved layout: chunk c of a 4-row batch = one 128-byte line
            return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(buf_rsrc(M + rb * 16), (c * 16 + q) * 8, 0, 0));
        }
        const int mk = min(qk, (int)(r1 - 1 - rb));
        const int sv = min(4 * c + qs, nd - 1);
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(buf_rsrc(M + rb), (sv * (int)rows + mk) * 8, 0, 0));
    };
    auto load_x = [&](double2 (&x)[RW], long long rb) {
        const int kmax = (int)(r1 - 1 - rb);
        const __amdgpu_buffer_rsrc_t rt = buf_rsrc(Ts + rb * ld);
#pragma unroll
        for (int k = 0; k < RW; ++k)
            x[k] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rt, lob, min(k, kmax) * ldb, (MODE & 256) ? 2 : (MODE & 512) ? 1 : 0));
    };
    const long long step = (long long)W * RW;
    long long rb = r0 + (long long)wave * RW;
    double2 xn[RW];
    double m[NM];
    if (rb < r1) {
        load_x(xn, rb);
#pragma unroll
        for (int c = 0; c < NM; ++c) m[c] = load_m(rb, c);
    }
    __syncthreads();
    const double2 pconst = make_double2(1e-3, 2e-3);
    for (; rb < r1; rb += step) {
        double2 x[RW];
#pragma unroll
        for (int k = 0; k < RW; ++k) x[k] = xn[k];
        const long long rn = rb + step;
        const bool more = rn < r1;
        if (more) load_x(xn, rn);
        const int kmax = (int)min((long long)RW - 1, r1 - 1 - rb);
        double2 pa = (MODE & 2) ? pconst : sp[0][lane], pb = (MODE & 2) ? pconst : sp[1][lane];
#pragma unroll
        for (int c = 0; c < NM; ++c) {
            if (c < nch) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int s2 = 4 * c + 2 * h + 2;
                    if (MODE & 2) {
                        dp_half<MODE>(x, m[c], pa, pb, h);
                        continue;
                    }
                    const double2 qa = sp[s2 < NB ? s2 : 0][lane], qb = sp[s2 + 1 < NB ? s2 + 1 : 1][lane];
                    dp_half<MODE>(x, m[c], pa, pb, h);
                    pa = qa;
                    pb = qb;
                }
            }
            if (more && !(MODE & 1)) m[c] = load_m(rn, c);
        }
        const __amdgpu_buffer_rsrc_t ro = buf_rsrc(Tos + rb * ld);
#pragma unroll
        for (int k = 0; k < RW; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, x[k]), ro, lob, min(k, kmax) * ldb, SA);
    }
}

__global__ void k_fill(double *a, long long n, double v)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        a[i] = v * (1.0 + 1e-3 * (double)(i % 977));
}

template <int MODE>
static int run_mode(double *T, double *P, double *M, long long rows, long long ld, int ncu, hipEvent_t e0,
                    hipEvent_t e1)
{
    const int ns = (int)((ld + 127) / 128);
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void *)&k_probe<MODE>, 512, 0));
    long long nrun = (long long)ncu * bpc / ns;
    if (nrun < 1) nrun = 1;
    long long run = (rows + nrun - 1) / nrun;
    run = (run + 3) / 4 * 4;
    nrun = (rows + run - 1) / run;
    std::vector<float> ms;
    for (int it = 0; it < 12; ++it) {
        CK(hipEventRecord(e0, 0));
        const long long nt = nrun * ns, gx = (MODE & 128) ? (nt + 7) / 8 * 8 : nt;
        hipLaunchKernelGGL(k_probe<MODE>, dim3((unsigned)gx), dim3(512), 0, 0, T, P, M, ld, rows, ns, run, 64, (int)nt);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t = 0.f;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (it >= 3) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double us = ms[ms.size() / 2] * 1e3;
    const double bytes = 8.0 * (2.0 * rows * (ld - 127) + 64.0 * (ld - 127) + 64.0 * rows);
    std::printf("{\"mode\": %d, \"workgroups_per_cu\": %d, \"grid\": %lld, \"us\": %.1f, \"GBps\": %.0f}\n", MODE, bpc,
                nrun * ns, us, bytes / us / 1e3);
    std::fflush(stdout);
    return 0;
}

int main()
{
    const long long rows = 32769, ld = 8320, n = rows * ld;
    double *T = nullptr, *P = nullptr, *M = nullptr;
    CK(hipMalloc(&T, n * 8));
    CK(hipMalloc(&P, 64 * ld * 8));
    CK(hipMalloc(&M, (64 * (rows + 8)) * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, T, n, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, P, 64 * ld, 1e-3);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, M, 64 * (rows + 8), 1e-3);
    CK(hipDeviceSynchronize());
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int rc = 0;
    rc |= run_mode<0>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<1>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<2>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<4>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<3>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<7>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<8>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<16>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<1024>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<1024 + 32>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<1024>(T, P, M, rows, ld, ncu, e0, e1);
    rc |= run_mode<0>(T, P, M, rows, ld, ncu, e0, e1);
    return rc;
}

// f64 matrix-core probe for the rank-64 elimination (k_sweep_*):
//   T[i][j] <- T[i][j] - sum_s M[i][s] P[s][j], one rounding per pivot s in
//   order (the reference's row operations, tableau.py:269-280; upd() in
//   kernels.hip: x = fma(-m, p, x)).
// (1) exactness: does a chain of v_mfma_f64_16x16x4_f64 (A = -M, B = P, four
//     pivots per instruction) give, for every element, exactly the sequential
//     fma chain?  Checked on the host against std::fma in pivot order, and
//     against a per-instruction "four products summed, one rounding" model;
//     integer-valued data (exact under any order) validates the operand
//     layout first.
// (2) rates: f64 FMAs per second of MFMA-only, VALU-only (v_fma_f64) and both
//     interleaved in one wave (independent), whole GPU.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_probe scripts/mfma_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int K = 64;   // pivots

// one wave per tile: A (16 x K, row-major), B (K x 16), C (16 x 16) of tile
// blockIdx.x; D out in the assumed layout: lane l, register r holds
// D[4 (l / 16) + r][l % 16]
__global__ void __launch_bounds__(64) tile(const double *A, const double *B, const double *C, double *D)
{
    const int l = threadIdx.x, t = blockIdx.x;
    const double *a = A + (size_t)t * 16 * K, *b = B + (size_t)t * K * 16, *c = C + (size_t)t * 256;
    d4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = c[(4 * (l / 16) + r) * 16 + l % 16];
    for (int k0 = 0; k0 < K; k0 += 4) {
        // A operand: lane l holds A[l % 16][k0 + l / 16]; B: B[k0 + l / 16][l % 16]
        const double av = a[(l % 16) * K + k0 + l / 16];
        const double bv = b[(k0 + l / 16) * 16 + l % 16];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) D[(size_t)t * 256 + (4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}

// rates: REPS x (independent chains) per wave
#define REPS 512
__global__ void __launch_bounds__(256) rate_mfma(double *out, const double *in)
{
    const int l = threadIdx.x;
    d4 a0 = {in[l], in[l] + 1, in[l] + 2, in[l] + 3}, a1 = a0 + 1.0, a2 = a0 + 2.0, a3 = a0 + 3.0;
    const double x = in[64 + (l & 63)], y = in[128 + (l & 63)];
    for (int r = 0; r < REPS; ++r) {
        a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
    }
    const d4 s = a0 + a1 + a2 + a3;
    out[blockIdx.x * 256 + l] = s[0] + s[1] + s[2] + s[3];
}
__global__ void __launch_bounds__(256) rate_valu(double *out, const double *in)
{
    const int l = threadIdx.x;
    double v[8];
    for (int k = 0; k < 8; ++k) v[k] = in[l] + k;
    const double x = in[64 + (l & 63)], y = in[128 + (l & 63)];
    for (int r = 0; r < REPS; ++r) {
        // 64 FMAs per lane = the FMAs of 4 MFMAs spread over 64 lanes
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[k]) : "v"(x), "v"(y));
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += v[k];
    out[blockIdx.x * 256 + l] = s;
}
__global__ void __launch_bounds__(256) rate_both(double *out, const double *in)
{
    const int l = threadIdx.x;
    d4 a0 = {in[l], in[l] + 1, in[l] + 2, in[l] + 3}, a1 = a0 + 1.0, a2 = a0 + 2.0, a3 = a0 + 3.0;
    double v[8];
    for (int k = 0; k < 8; ++k) v[k] = in[l] + k;
    const double x = in[64 + (l & 63)], y = in[128 + (l & 63)];
    for (int r = 0; r < REPS; ++r) {
        a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[k]) : "v"(x), "v"(y));
        a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a1, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[k]) : "v"(x), "v"(y));
        a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a2, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[k]) : "v"(x), "v"(y));
        a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a3, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[k]) : "v"(x), "v"(y));
    }
    const d4 s4 = a0 + a1 + a2 + a3;
    double s = s4[0] + s4[1] + s4[2] + s4[3];
    for (int k = 0; k < 8; ++k) s += v[k];
    out[blockIdx.x * 256 + l] = s;
}

static double rnd(std::mt19937_64 &g, bool integers)
{
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    if (integers) return std::floor(u(g) * 64.0);
    std::uniform_int_distribution<int> e(-8, 8);
    return std::ldexp(u(g), e(g));
}

int main()
{
    const int NT = 4096;   // tiles
    std::vector<double> A((size_t)NT * 16 * K), B((size_t)NT * K * 16), C((size_t)NT * 256), D(C.size());
    double *dA, *dB, *dC, *dD;
    CHK(hipMalloc(&dA, A.size() * 8));
    CHK(hipMalloc(&dB, B.size() * 8));
    CHK(hipMalloc(&dC, C.size() * 8));
    CHK(hipMalloc(&dD, D.size() * 8));
    for (int pass = 0; pass < 2; ++pass) {
        const bool ints = pass == 0;
        std::mt19937_64 g(1234 + pass);
        for (auto &x : A) x = -rnd(g, ints);          // A = -M
        for (auto &x : B) x = rnd(g, ints);
        for (auto &x : C) x = rnd(g, ints);
        CHK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
        CHK(hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice));
        CHK(hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(tile, dim3(NT), dim3(64), 0, 0, dA, dB, dC, dD);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost));
        long long seq_bad = 0, dot4_bad = 0, n = 0;
        for (int t = 0; t < NT; ++t)
            for (int i = 0; i < 16; ++i)
                for (int j = 0; j < 16; ++j) {
                    const double *a = &A[(size_t)t * 16 * K + i * K];
                    const double *b = &B[(size_t)t * K * 16 + j];
                    double x = C[(size_t)t * 256 + i * 16 + j], y = x;
                    for (int s = 0; s < K; ++s) x = std::fma(a[s], b[s * 16], x);
                    for (int s = 0; s < K; s += 4) {
                        long double p = (long double)a[s] * b[s * 16] + (long double)a[s + 1] * b[(s + 1) * 16] +
                                        (long double)a[s + 2] * b[(s + 2) * 16] +
                                        (long double)a[s + 3] * b[(s + 3) * 16];
                        y = (double)((long double)y + p);
                    }
                    const double d = D[(size_t)t * 256 + i * 16 + j];
                    seq_bad += std::memcmp(&d, &x, 8) != 0;
                    dot4_bad += std::memcmp(&d, &y, 8) != 0;
                    ++n;
                }
        printf("{\"probe\": \"mfma_f64_exactness\", \"data\": \"%s\", \"elements\": %lld, "
               "\"differ_from_sequential_fma\": %lld, \"differ_from_dot4_model\": %lld}\n",
               ints ? "integers (layout check)" : "random doubles 2^-8..2^8", n, seq_bad, dot4_bad);
    }
    // rates
    const int blocks = 2048;   // 8 waves per CU x 256 CUs
    double *out, *in;
    CHK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    CHK(hipMalloc(&in, 4096 * 8));
    std::vector<double> hin(4096, 1e-3);
    CHK(hipMemcpy(in, hin.data(), hin.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto run = [&](const char *name, void (*k)(double *, const double *), double fma_per_wave_rep) {
        for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, in);
        CHK(hipEventRecord(e0));
        for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, in);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        const double fmas = 5.0 * blocks * 4 * REPS * fma_per_wave_rep;
        printf("{\"probe\": \"rate\", \"kernel\": \"%s\", \"ms\": %.3f, \"TFMA_s\": %.2f, \"TFLOP_s\": %.2f}\n", name,
               ms / 5, fmas / (ms * 1e-3) / 1e12, 2 * fmas / (ms * 1e-3) / 1e12);
    };
    run("mfma_f64_16x16x4 (4 chains)", rate_mfma, 4 * 1024.0);
    run("v_fma_f64 (8 chains)", rate_valu, 64 * 64.0);
    run("both interleaved", rate_both, 4 * 1024.0 + 32 * 64.0);
    return 0;
}

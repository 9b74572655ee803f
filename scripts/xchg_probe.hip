// Hand-off latency probe for the one-XCD selection's exchanges: two
// single-wave blocks on one XCD ping-pong a tagged 8-byte word through L2
// (block 0 stores round r, block 1 polls for it and answers, block 0 polls
// for the answer); half the round trip is the one-way hand-off latency.
// Variants: store scope (workgroup = plain store kept in L2 / agent =
// write-through), drain after the store or not, sleep between polls, and
// `crowd` other blocks polling the same lines meanwhile (as the 64 blocks of
// an exchange do).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/xchg_probe scripts/xchg_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
#define NR 256

template <int SCOPE>
__device__ __forceinline__ void st(u64 *p, u64 v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, SCOPE);
}
__device__ __forceinline__ u64 ld(const u64 *p)
{
    return __hip_atomic_load(const_cast<u64 *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int SCOPE, bool DRAIN, int SLEEP>
__global__ void __launch_bounds__(64) pingpong(u64 *buf, u64 *cyc, int crowd, int base)
{
    if (blockIdx.x & 7u) return;
    const unsigned b = blockIdx.x >> 3;
    const int lane = threadIdx.x;
    u64 *ping = buf, *pong = buf + 64, *stop = buf + 128;
    if (b == 0) {
        const u64 t0 = __builtin_amdgcn_s_memtime();
        for (int r = 1; r <= NR; ++r) {
            if (lane == 0) st<SCOPE>(ping, (u64)(base + r));
            if (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            while (!__all(ld(pong) == (u64)(base + r))) {
                if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
            }
        }
        const u64 t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            cyc[0] = t1 - t0;
            st<__HIP_MEMORY_SCOPE_AGENT>(stop, (u64)base);
        }
    } else if (b == 1) {
        for (int r = 1; r <= NR; ++r) {
            while (!__all(ld(ping) == (u64)(base + r))) {
                if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
            }
            if (lane == 0) st<SCOPE>(pong, (u64)(base + r));
            if (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else if ((int)b < 2 + crowd) {
        // bystanders: poll 9 granule rows of 512 B next to the words, as an
        // exchange's blocks do, until block 0 is done
        const u64 *rows = buf + 256;
        for (;;) {
            u64 acc = 0;
#pragma unroll
            for (int g = 0; g < 9; ++g) acc += ld(rows + g * 64 + lane);
            if (__all(ld(stop) == (u64)base) || acc == 12345) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
}


// an exchange as k_sel runs it: every block publishes NG granules (lanes < NG,
// granule g of block b at [g * 64 + b]) and polls until it has every block's;
// round r's tag is base + r.  100 MHz stamps of each block's publication
// and detection, per round.
template <int NG, int SLEEP, int FETCH>
__global__ void __launch_bounds__(64) gatherp(u64 *reg, u64 *stamps, int G, int base)
{
    if (blockIdx.x & 7u) return;
    const unsigned b = blockIdx.x >> 3;
    const int lane = threadIdx.x;
    if ((int)b >= G) return;
    for (int r = 1; r <= NR; ++r) {
        // two regions in turn (as k_sel's ratio / row-0 summaries): a block
        // can be one exchange ahead of another, never two
        u64 *rg = reg + (r & 1) * 1024;
        const u64 *p = rg + min((unsigned)lane, (unsigned)G - 1);
        const u64 tag = (u64)(base + r) << 32;
        if (lane < NG + FETCH) st<__HIP_MEMORY_SCOPE_WORKGROUP>(&rg[lane * 64 + b], tag | (unsigned)(b * 16 + lane));
        const u64 tp = __builtin_amdgcn_s_memrealtime();
        u64 v[NG];
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int g = 0; g < NG; ++g) v[g] = ld(p + g * 64);
#pragma unroll
            for (int g = 0; g < NG; ++g) ok = ok && (v[g] >> 32) == (tag >> 32);
            if (__all(ok)) break;
            if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
        }
        if (FETCH) {
            // the winner's other granules, one load (lanes 0..FETCH-1)
            const unsigned bw = (unsigned)(v[0] & 63u) % (unsigned)G;
            for (;;) {
                const u64 f = ld(rg + (NG + min(lane, FETCH - 1)) * 64 + bw);
                if (__all((f >> 32) == (tag >> 32))) break;
            }
        }
        const u64 ts = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            stamps[(r * 64 + b) * 2] = tp;
            stamps[(r * 64 + b) * 2 + 1] = ts;
        }
    }
}

int main()
{
    u64 *buf, *cyc;
    hipMalloc(&buf, 4096 * sizeof(u64));
    hipMalloc(&cyc, 64 * sizeof(u64));
    hipMemset(buf, 0, 4096 * sizeof(u64));
    int base = 0;
    auto run = [&](auto kern, const char *name, int crowd) {
        double best = 1e30, sum = 0;
        for (int rep = 0; rep < 5; ++rep) {
            base += 1000;
            hipLaunchKernelGGL(kern, dim3(8 * 64), dim3(64), 0, 0, buf, cyc, crowd, base);
            hipDeviceSynchronize();
            u64 c = 0;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double oneway = c / (2.0 * NR);
            if (rep > 0) {
                sum += oneway;
                best = oneway < best ? oneway : best;
            }
        }
        printf("%-44s crowd %2d: one-way %6.0f cycles (best %6.0f)\n", name, crowd, sum / 4, best);
    };
    for (int crowd : {0}) {
        run(pingpong<__HIP_MEMORY_SCOPE_WORKGROUP, false, 1>, "workgroup store, sleep 1", crowd);
        run(pingpong<__HIP_MEMORY_SCOPE_WORKGROUP, false, 0>, "workgroup store, no sleep", crowd);
        run(pingpong<__HIP_MEMORY_SCOPE_WORKGROUP, true, 1>, "workgroup store + drain, sleep 1", crowd);
        run(pingpong<__HIP_MEMORY_SCOPE_AGENT, false, 1>, "agent store, sleep 1", crowd);
        run(pingpong<__HIP_MEMORY_SCOPE_AGENT, true, 1>, "agent store + drain, sleep 1", crowd);
    }
    {
        u64 *stamps;
        hipMalloc(&stamps, (NR + 1) * 64 * 2 * sizeof(u64));
        std::vector<u64> h((NR + 1) * 64 * 2);
        auto grun = [&](auto kern, const char *name, int G) {
            base += 1000;
            hipMemset(buf, 0, 4096 * sizeof(u64));
            hipLaunchKernelGGL(kern, dim3(8 * 64), dim3(64), 0, 0, buf, stamps, G, base);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
            double seen_mean = 0, seen_min = 0, seen_max = 0, spread = 0;
            int n = 0;
            for (int r = 8; r <= NR; ++r) {
                u64 pmax = 0, pmin = ~0ull;
                for (int b = 0; b < G; ++b) {
                    pmax = std::max(pmax, h[(r * 64 + b) * 2]);
                    pmin = std::min(pmin, h[(r * 64 + b) * 2]);
                }
                double mn = 1e30, mx = 0, sm = 0;
                for (int b = 0; b < G; ++b) {
                    const double d = (double)(long long)(h[(r * 64 + b) * 2 + 1] - pmax) * 10.0;
                    mn = std::min(mn, d);
                    mx = std::max(mx, d);
                    sm += d;
                }
                seen_mean += sm / G;
                seen_min += mn;
                seen_max += mx;
                spread += (double)(pmax - pmin) * 10.0;
                ++n;
            }
            printf("%-36s G %2d: after the last publication: min %5.0f mean %5.0f max %5.0f ns; publication spread %5.0f ns\n",
                   name, G, seen_min / n, seen_mean / n, seen_max / n, spread / n);
        };
        for (int G : {64}) {
            grun(gatherp<9, 1, 0>, "gather 9 granules", G);
            grun(gatherp<7, 1, 0>, "gather 7 granules", G);
            grun(gatherp<3, 1, 0>, "gather 3 granules", G);
            grun(gatherp<3, 1, 4>, "gather 3 + fetch 4 of one block", G);
            grun(gatherp<2, 1, 0>, "gather 2 granules", G);
            grun(gatherp<1, 1, 0>, "gather 1 granule", G);
        }
    }
    return 0;
}

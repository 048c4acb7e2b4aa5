// Streaming probe for the bucket aggregation's access pattern (not product code): 256 workgroups of
// 1024 threads, workgroup b streams "bucket" b = 256 regions of ~5.3 K 16-byte records (80 % of a
// region's capacity), waves taking chunks of 64 * U records in turn, D chunks in flight per wave.
// Prints GB/s of records read per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
#define GAS __attribute__((address_space(1)))
constexpr int NB = 256, NR = 256;
struct Args { const u64x2 *pool; const uint32_t *rn; uint32_t cap; unsigned long long *sink; };

template <int U, int D>
__global__ __launch_bounds__(1024, 1) void k_stream(Args A) {
    __shared__ uint32_t s_cs[NR + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t b = blockIdx.x;
    constexpr uint32_t CH = 64u * U;
    if (tid == 0) {
        uint32_t run = 0;
        for (int r = 0; r < NR; ++r) { s_cs[r] = run; run += (A.rn[b * NR + r] + CH - 1) / CH; }
        s_cs[NR] = run;
    }
    __syncthreads();
    const uint32_t NC = s_cs[NR];
    const GAS u64x2 *pool = (const GAS u64x2 *)A.pool + (uint64_t)b * NR * A.cap;
    uint64_t acc = 0;
    u64x2 buf[D][U];
    uint32_t rr = 0;
    auto pos = [&](uint32_t k, uint32_t &r, uint32_t &n) -> const GAS u64x2 * {
        while (s_cs[r + 1] <= k) ++r;
        n = A.rn[b * NR + r];
        return pool + (uint64_t)r * A.cap + (k - s_cs[r]) * CH;
    };
    // prologue: D chunks
    uint32_t k0 = wv;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const uint32_t k = k0 + d * 16u;
        if (k < NC) {
            uint32_t n; const GAS u64x2 *src = pos(k, rr, n);
            const uint32_t off = (k - s_cs[rr]) * CH;
#pragma unroll
            for (int u = 0; u < U; ++u) buf[d][u] = __builtin_nontemporal_load(src + min(64u * u + lane, n - 1 - off));
        }
    }
    for (uint32_t k = k0; k < NC; k += 16u * D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t kc = k + d * 16u;
            if (kc >= NC) break;
#pragma unroll
            for (int u = 0; u < U; ++u) acc += buf[d][u].x ^ buf[d][u].y;
            const uint32_t kn = kc + 16u * D;
            if (kn < NC) {
                uint32_t n; const GAS u64x2 *src = pos(kn, rr, n);
                const uint32_t off = (kn - s_cs[rr]) * CH;
#pragma unroll
                for (int u = 0; u < U; ++u) buf[d][u] = __builtin_nontemporal_load(src + min(64u * u + lane, n - 1 - off));
            }
        }
    }
    if (acc == 0x123456789ull) atomicAdd(A.sink, 1ull);
}

template <int U, int D>
double run(const Args &A, uint64_t bytes) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((k_stream<U, D>), dim3(NB), dim3(1024), 0, 0, A);
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k_stream<U, D>), dim3(NB), dim3(1024), 0, 0, A);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return bytes * 5.0 / (ms / 1e3) / 1e9;
}

int main() {
    const uint32_t cap = 6656;  // records per region (1.25 x the mean)
    std::vector<uint32_t> rn(NB * NR);
    uint64_t tot = 0;
    for (int i = 0; i < NB * NR; ++i) { rn[i] = 5325 + (uint32_t)((i * 2654435761u) % 600) - 300; tot += rn[i]; }
    Args A{};
    void *p; hipMalloc(&p, (size_t)NB * NR * cap * 16); hipMemset(p, 1, (size_t)NB * NR * cap * 16);
    uint32_t *drn; hipMalloc(&drn, rn.size() * 4); hipMemcpy(drn, rn.data(), rn.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&A.sink, 8);
    A.pool = (const u64x2 *)p; A.rn = drn; A.cap = cap;
    const uint64_t bytes = tot * 16;
    printf("records %llu (%.2f GB)\n", (unsigned long long)tot, bytes / 1e9);
    printf("U=8 D=2 (today): %.0f GB/s\n", run<8, 2>(A, bytes));
    printf("U=4 D=2: %.0f GB/s\n", run<4, 2>(A, bytes));
    printf("U=4 D=4: %.0f GB/s\n", run<4, 4>(A, bytes));
    printf("U=8 D=3: %.0f GB/s\n", run<8, 3>(A, bytes));
    printf("U=16 D=2: %.0f GB/s\n", run<16, 2>(A, bytes));
    printf("U=2 D=8: %.0f GB/s\n", run<2, 8>(A, bytes));
    return 0;
}

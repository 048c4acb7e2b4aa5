#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void k(uint32_t *out, int mode) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) buf[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const uint32_t off0 = mode == 2 ? threadIdx.x * 16 : threadIdx.x * 9 + 1;
    const uint32_t off = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)(buf + off0);
    u32x4 v;
    uint32_t w;
    if (mode != 1) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b32 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)" : "=v"(v), "=v"(w) : "v"(off) : "memory");
    } else {
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(*(uint64_t*)&v) : "v"(off) : "memory");
        v.z = 0; v.w = 0; w = 0;
    }
    out[threadIdx.x * 5 + 0] = v.x; out[threadIdx.x * 5 + 1] = v.y; out[threadIdx.x * 5 + 2] = v.z;
    out[threadIdx.x * 5 + 3] = v.w; out[threadIdx.x * 5 + 4] = w;
}
int main() {
    uint32_t *d; hipMalloc(&d, 64 * 5 * 4);
    uint32_t h[320];
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipError_t e = hipDeviceSynchronize();
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l) {
            uint32_t off = mode == 2 ? l * 16 : l * 9 + 1;
            int nw = mode != 1 ? 5 : 2;
            for (int j = 0; j < nw; ++j) {
                uint32_t exp = 0;
                for (int b = 0; b < 4; ++b) exp |= (uint32_t)(uint8_t)((off + 4 * j + b) * 7 + 3) << (8 * b);
                if (h[l * 5 + j] != exp) { if (bad < 5) printf("mode %d lane %d word %d got %08x exp %08x\n", mode, l, j, h[l*5+j], exp); ++bad; }
            }
        }
        printf("mode %d: err=%s bad=%d\n", mode, hipGetErrorString(e), bad);
    }
    return 0;
}

// Probe: LDS placement of global_load_lds_dwordx3 (lane stride 12 or 16 B?).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(const uint8_t *src, uint8_t *dst) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 16 + 64];
    for (int i = threadIdx.x; i < 64 * 16 + 64; i += 64) lds[i] = 0xEE;
    __syncthreads();
    const uint8_t *a = src + threadIdx.x * 32;  // lane l reads bytes [32l, 32l+12)
    __builtin_amdgcn_global_load_lds(a, (__attribute__((address_space(3))) void *)lds, 12, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 16 + 64; i += 64) dst[i] = lds[i];
}

int main() {
    uint8_t h[64 * 32];
    for (int i = 0; i < 64 * 32; ++i) h[i] = (uint8_t)i;
    uint8_t *s, *d;
    hipMalloc(&s, sizeof h);
    hipMalloc(&d, 64 * 16 + 64);
    hipMemcpy(s, h, sizeof h, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(s, d);
    uint8_t o[64 * 16 + 64];
    hipMemcpy(o, d, sizeof o, hipMemcpyDeviceToHost);
    for (int r = 0; r < 8; ++r) {
        for (int c = 0; c < 16; ++c) printf("%02x ", o[r * 16 + c]);
        printf("\n");
    }
    // lane 5 expected source bytes 160..171 (0xa0..0xab)
    printf("stride12: lane5@60 = %02x, stride16: lane5@80 = %02x\n", o[60], o[80]);
    return 0;
}

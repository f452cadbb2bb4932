// Micro-benchmark (tools only): the C2 walker's memory pattern - one wave per
// 64-pair pack, ~160 row phases, two 12-byte segment loads per lane and
// phase (the current block and its left neighbour), lanes scattered over the
// row's 8 blocks - through (A) LDS-DMA (global_load_lds_dwordx3 into a
// 4-slot window per block, counted vmcnt, ds_read_b128: the shipped walker's
// way) and (B) plain global_load_dwordx3 into a 4-deep VGPR ring with the
// same counted waits.  Prints the kernel time of each over 1,563 waves.
//   hipcc --offload-arch=gfx950 -O3 walk_load_rate.hip -o walk_load_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t kRows = 150, kBlocks = 8, kSeg = 12, kPack = 64;
constexpr uint64_t kRs = (uint64_t)kBlocks * kPack * kSeg;  // 6144 B per pack row
constexpr uint64_t kPackBytes = kRows * kRs;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ uint32_t block_of(uint32_t lane, uint32_t row) {
    // a path from the last block (row 150) to block 0 (row 1), lanes spread
    const uint32_t b = (row * kBlocks + (lane * 7u) % 19u) / (kRows + 1);
    return b < kBlocks ? b : kBlocks - 1;
}

template <int kMode>
__global__ __launch_bounds__(128) void walk_loads(const uint8_t *__restrict__ mask, uint32_t *out,
                                                  uint32_t n_packs) {
    __shared__ __attribute__((aligned(16))) uint8_t win_all[2][2 * 4 * 1024];
    const uint32_t wave = blockIdx.x * 2 + threadIdx.x / 64, lane = threadIdx.x & 63u;
    if (wave >= n_packs) return;
    const uint8_t *base = mask + (uint64_t)wave * kPackBytes + lane * kSeg;
    uint32_t acc = 0;
    if constexpr (kMode == 0) {
        __attribute__((address_space(3))) uint8_t *win =
            (__attribute__((address_space(3))) uint8_t *)win_all[threadIdx.x / 64];
        auto dma = [&](uint32_t w, uint32_t s, uint32_t row) {
            const uint32_t b = block_of(lane, row);
            const uint8_t *a = base + (uint64_t)(row - 1) * kRs + (uint64_t)(w ? (b ? b - 1 : 0) : b) * kPack * kSeg;
            __builtin_amdgcn_global_load_lds(a, (__attribute__((address_space(3))) void *)(win + w * 4096 + s * 1024), 12, 0, 0);
        };
        for (uint32_t s = 0; s < 4; ++s) { dma(0, s, kRows - s); dma(1, s, kRows - s); }
        for (uint32_t r0 = kRows; r0 > 4; r0 -= 4) {
#pragma unroll
            for (uint32_t s = 0; s < 4; ++s) {
                const uint32_t addr = (uint32_t)(uintptr_t)(win + s * 1024) + lane * 16u;
                u32x4 v;
                asm volatile("s_waitcnt vmcnt(6)\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(v) : "v"(addr) : "memory");
                acc ^= v.x + v.y + v.z;
                const int32_t row = (int32_t)r0 - (int32_t)s - 4;  // rows below 1 load row 1
                dma(0, s, row > 0 ? (uint32_t)row : 1u);
                dma(1, s, row > 0 ? (uint32_t)row : 1u);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
    } else {
        u32x3 ring0[4], ring1[4];
        auto ld = [&](u32x3 &dst0, u32x3 &dst1, uint32_t row) {
            const uint32_t b = block_of(lane, row);
            const uint8_t *a0 = base + (uint64_t)(row - 1) * kRs + (uint64_t)b * kPack * kSeg;
            const uint8_t *a1 = base + (uint64_t)(row - 1) * kRs + (uint64_t)(b ? b - 1 : 0) * kPack * kSeg;
            asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(dst0) : "v"(a0) : "memory");
            asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(dst1) : "v"(a1) : "memory");
        };
#pragma unroll
        for (uint32_t s = 0; s < 4; ++s) ld(ring0[s], ring1[s], kRows - s);
        for (uint32_t r0 = kRows; r0 > 4; r0 -= 4) {
#pragma unroll
            for (uint32_t s = 0; s < 4; ++s) {
                asm volatile("s_waitcnt vmcnt(6)" : "+v"(ring0[s]), "+v"(ring1[s]) : : "memory");
                acc ^= ring0[s].x + ring0[s].y + ring0[s].z + ring1[s].x;
                const int32_t row = (int32_t)r0 - (int32_t)s - 4;
                ld(ring0[s], ring1[s], row > 0 ? (uint32_t)row : 1u);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(ring0[0]), "+v"(ring1[0]) : : "memory");
    }
    out[wave * 64 + lane] = acc;
}

int main() {
    const uint32_t n_packs = 1563;
    uint8_t *mask;
    uint32_t *out;
    hipMalloc(&mask, (size_t)n_packs * kPackBytes + 4096);
    hipMemset(mask, 1, (size_t)n_packs * kPackBytes + 4096);
    hipMalloc(&out, n_packs * 64 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 4; ++rep) {
            hipEventRecord(a);
            if (mode == 0) walk_loads<0><<<(n_packs + 1) / 2, 128>>>(mask, out, n_packs);
            else walk_loads<1><<<(n_packs + 1) / 2, 128>>>(mask, out, n_packs);
            hipEventRecord(b);
            if (hipEventSynchronize(b) != hipSuccess || hipGetLastError() != hipSuccess) {
                fprintf(stderr, "kernel failed\n");
                return 1;
            }
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("{\"mode\": \"%s\", \"ms\": %.4f}\n", mode ? "vgpr" : "lds_dma", ms);
        }
    }
    return 0;
}

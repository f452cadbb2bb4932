// VALU issue-rate microbenchmark (gfx950): cycles per wave64 instruction for
// the instruction classes the fill kernels use, at 1..8 waves per SIMD.
// Each lane runs 8 independent chains of one instruction (inline asm, so the
// compiler cannot fold them); time per instruction = elapsed / (instructions
// per SIMD).  Build: hipcc -O3 --offload-arch=gfx950 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define OP2(name, ins)                                                                   \
    struct name {                                                                        \
        static constexpr const char *s = ins;                                            \
        __device__ static void run(uint32_t (&a)[8], uint32_t b) {                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i)                                \
                asm volatile(ins " %0, %0, %1" : "+v"(a[i]) : "v"(b));                   \
        }                                                                                \
    };
#define OP3(name, ins)                                                                   \
    struct name {                                                                        \
        static constexpr const char *s = ins;                                            \
        __device__ static void run(uint32_t (&a)[8], uint32_t b) {                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i)                                \
                asm volatile(ins " %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));               \
        }                                                                                \
    };

OP2(PkMaxI16, "v_pk_max_i16")
OP2(PkAddU16, "v_pk_add_u16")
OP2(SubU32, "v_sub_u32")
OP2(AndB32, "v_and_b32")
OP2(LshlB32, "v_lshlrev_b32")
OP2(MinU32, "v_min_u32")
OP2(MaxI16, "v_max_i16")
OP2(SubU16, "v_sub_u16")
OP2(MaxU32, "v_max_u32")
OP3(LshlOr, "v_lshl_or_b32")
OP3(Or3, "v_or3_b32")
OP3(Xad, "v_xad_u32")
struct MadU64 {
    static constexpr const char *s = "v_mad_u64_u32";
    __device__ static void run(uint32_t (&a)[8], uint32_t b) {
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {
            uint64_t acc = ((uint64_t)a[2 * i + 1] << 32) | a[2 * i];
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(b), "v"(b));
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(b), "v"(b));
            a[2 * i] = (uint32_t)acc; a[2 * i + 1] = (uint32_t)(acc >> 32);
        }
    }
};
struct MovDpp {
    static constexpr const char *s = "v_mov_b32_dpp row_shr:1";
    __device__ static void run(uint32_t (&a)[8], uint32_t b) {
        _Pragma("unroll") for (int i = 0; i < 8; ++i)
            asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 1) % 8]));
    }
};
OP2(PkSubI16, "v_pk_sub_i16")
OP2(PkMinU16, "v_pk_min_u16")
OP2(MaxI32, "v_max_i32")
OP2(AddU32, "v_add_u32")
OP2(XorB32, "v_xor_b32")
OP2(MaxF32, "v_max_f32")
OP2(AddF32, "v_add_f32")
OP3(Max3I32, "v_max3_i32")
OP3(Add3U32, "v_add3_u32")
OP3(PermB32, "v_perm_b32")
OP3(BfiB32, "v_bfi_b32")
OP3(Max3F32, "v_max3_f32")
OP3(AndOrB32, "v_and_or_b32")
OP3(Max3I16, "v_max3_i16")

constexpr int kIters = 4096;

template <class Op>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i);
    const uint32_t b = seed ^ blockIdx.x;
    for (int it = 0; it < kIters; ++it) {
        Op::run(a, b);
        Op::run(a, b);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= a[i];
    if (s == 0x12345678u) out[0] = s;
}

template <class Op>
static void bench(uint32_t *out, hipEvent_t e0, hipEvent_t e1, int cus) {
    for (int w : {1, 2, 4, 8}) {
        const dim3 grid(cus * w);  // 256-thread blocks: one wave per SIMD each
        k<Op><<<grid, 256>>>(out, 3);
        hipEventRecord(e0);
        k<Op><<<grid, 256>>>(out, 5);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double per_simd = (double)w * kIters * 16;  // wave-instructions per SIMD
        printf("%-14s waves/SIMD=%d  %.3f ms  %.2f ns/instr/SIMD\n", Op::s, w, ms,
               ms * 1e6 / per_simd);
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("CUs=%d clock=%d kHz\n", cus, p.clockRate);
    uint32_t *out;
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    bench<PkMaxI16>(out, e0, e1, cus);
    bench<PkAddU16>(out, e0, e1, cus);
    bench<SubU32>(out, e0, e1, cus);
    bench<AndB32>(out, e0, e1, cus);
    bench<LshlB32>(out, e0, e1, cus);
    bench<MinU32>(out, e0, e1, cus);
    bench<MaxU32>(out, e0, e1, cus);
    bench<MaxI16>(out, e0, e1, cus);
    bench<SubU16>(out, e0, e1, cus);
    bench<LshlOr>(out, e0, e1, cus);
    bench<Or3>(out, e0, e1, cus);
    bench<Xad>(out, e0, e1, cus);
    bench<MadU64>(out, e0, e1, cus);
    bench<MovDpp>(out, e0, e1, cus);
    bench<PkSubI16>(out, e0, e1, cus);
    bench<PkMinU16>(out, e0, e1, cus);
    bench<MaxI32>(out, e0, e1, cus);
    bench<AddU32>(out, e0, e1, cus);
    bench<XorB32>(out, e0, e1, cus);
    bench<MaxF32>(out, e0, e1, cus);
    bench<AddF32>(out, e0, e1, cus);
    bench<Max3I32>(out, e0, e1, cus);
    bench<Add3U32>(out, e0, e1, cus);
    bench<PermB32>(out, e0, e1, cus);
    bench<BfiB32>(out, e0, e1, cus);
    bench<Max3F32>(out, e0, e1, cus);
    bench<AndOrB32>(out, e0, e1, cus);
    bench<Max3I16>(out, e0, e1, cus);
    return 0;
}

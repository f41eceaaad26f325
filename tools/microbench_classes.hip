// microbench_classes.hip -- issue cost of the instruction classes the flat tracer executes
// (tools/cycle_attrib.py weights the kernel's measured instruction mix with these):
// one kernel per instruction form, 8 independent chains per wave, ITERS x 8 instructions.
// Timed with HIP events at 8 waves per SIMD (throughput: the SIMD's pipe) and at 1 wave per SIMD
// (one wave's issue interval), each relative to v_mul_f32; run it under rocprofv3 --pmc to get
// SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU per form (the counter's quad-cycles per instruction).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_classes.hip -o tools/microbench_classes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define ITERS 2048

typedef float v2f __attribute__((ext_vector_type(2)));

// eight independent chains of one instruction form on 32-bit VGPRs
#define K32(NAME, FMT)                                                                         \
    __global__ void NAME(float* out, float s) {                                                \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
              a6 = a0 + 6, a7 = a0 + 7;                                                        \
        for (int i = 0; i < ITERS; i++) {                                                      \
            asm volatile(FMT("%0") FMT("%1") FMT("%2") FMT("%3") FMT("%4") FMT("%5") FMT("%6")  \
                             FMT("%7")                                                         \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),          \
                           "+v"(a6), "+v"(a7)                                                  \
                         : "v"(s)                                                              \
                         : "vcc");                                                             \
        }                                                                                      \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;    \
    }
// the same on 64-bit VGPR pairs
#define K64(NAME, FMT)                                                                         \
    __global__ void NAME(float* out, float s) {                                                \
        double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,           \
               a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, sv = s;                                  \
        for (int i = 0; i < ITERS; i++) {                                                      \
            asm volatile(FMT("%0") FMT("%1") FMT("%2") FMT("%3") FMT("%4") FMT("%5") FMT("%6")  \
                             FMT("%7")                                                         \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),          \
                           "+v"(a6), "+v"(a7)                                                  \
                         : "v"(sv)                                                             \
                         : "vcc");                                                             \
        }                                                                                      \
        out[blockIdx.x * blockDim.x + threadIdx.x] =                                           \
            (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);                                    \
    }
// packed fp32 on v2f pairs
#define KPK(NAME, FMT)                                                                         \
    __global__ void NAME(float* out, float s) {                                                \
        v2f a0 = {float(threadIdx.x), 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
            a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, sv = {s, s};                                \
        for (int i = 0; i < ITERS; i++) {                                                      \
            asm volatile(FMT("%0") FMT("%1") FMT("%2") FMT("%3") FMT("%4") FMT("%5") FMT("%6")  \
                             FMT("%7")                                                         \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),          \
                           "+v"(a6), "+v"(a7)                                                  \
                         : "v"(sv));                                                           \
        }                                                                                      \
        v2f t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                         \
        out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;                                \
    }

#define F_MUL(r) "v_mul_f32 " r ", " r ", %8\n"
#define F_FMA(r) "v_fma_f32 " r ", " r ", %8, %8\n"
#define F_MOV(r) "v_mov_b32 " r ", %8\n"
#define F_CND(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define F_ADDU(r) "v_add_u32 " r ", " r ", %8\n"
#define F_MAX3(r) "v_max3_f32 " r ", " r ", %8, %8\n"
#define F_CMP(r) "v_cmp_lt_f32 vcc, " r ", %8\n"
#define F_SQRT(r) "v_sqrt_f32 " r ", " r "\n"
#define F_RCP(r) "v_rcp_f32 " r ", " r "\n"
#define F_DSC(r) "v_div_scale_f32 " r ", vcc, " r ", %8, " r "\n"
#define F_DFM(r) "v_div_fmas_f32 " r ", " r ", %8, %8\n"
#define F_DFX(r) "v_div_fixup_f32 " r ", " r ", %8, %8\n"
#define F_MULLO(r) "v_mul_lo_u32 " r ", " r ", %8\n"
#define F_MULHI(r) "v_mul_hi_u32 " r ", " r ", %8\n"
#define F_DPP(r) "v_add_u32_dpp " r ", " r ", " r " row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define F_MBCNT(r) "v_mbcnt_lo_u32_b32 " r ", %8, " r "\n"
#define F_BFE(r) "v_bfe_u32 " r ", " r ", 1, 5\n"
#define F_FMA64(r) "v_fma_f64 " r ", " r ", %8, %8\n"
#define F_MUL64(r) "v_mul_f64 " r ", " r ", %8\n"
#define F_ADD64(r) "v_add_f64 " r ", " r ", %8\n"
#define F_LSHL64(r) "v_lshl_add_u64 " r ", " r ", 1, " r "\n"
#define F_RCP64(r) "v_rcp_f64 " r ", " r "\n"
#define F_PKFMA(r) "v_pk_fma_f32 " r ", " r ", %8, %8\n"
#define F_PKMUL(r) "v_pk_mul_f32 " r ", " r ", %8\n"
#define F_PKADD(r) "v_pk_add_f32 " r ", " r ", %8\n"
#define F_FMAC(r) "v_fmac_f32 " r ", %8, %8\n"
#define F_MAX(r) "v_max_f32 " r ", " r ", %8\n"
#define F_AND(r) "v_and_b32 " r ", " r ", %8\n"
#define F_LSHL(r) "v_lshlrev_b32 " r ", 1, " r "\n"
#define F_ALIGN(r) "v_alignbit_b32 " r ", " r ", %8, 31\n"
#define F_MULE64(r) "v_mul_f32_e64 " r ", " r ", %8\n"
#define F_SUB(r) "v_sub_f32 " r ", " r ", %8\n"
#define F_ADDF(r) "v_add_f32 " r ", " r ", %8\n"
#define F_MIN(r) "v_min_f32 " r ", " r ", %8\n"
#define F_OR(r) "v_or_b32 " r ", " r ", %8\n"
#define F_XOR(r) "v_xor_b32 " r ", " r ", %8\n"
#define F_LSHLV(r) "v_lshlrev_b32 " r ", %8, " r "\n"
#define F_MULLIT(r) "v_mul_f32 " r ", 0x3f7fbe77, " r "\n"
#define F_MED3(r) "v_med3_f32 " r ", " r ", %8, %8\n"
#define F_CVTF32F64(r) "v_cvt_f32_f64 " r ", %9\n"
#define F_CMPVCND(r) "v_cmp_lt_f32 vcc, " r ", %8\n v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define F_CMPSCND(r) "v_cmp_lt_f32 s[20:21], " r ", %8\n v_cndmask_b32_e64 " r ", " r ", %8, s[20:21]\n"

K32(k_mul, F_MUL)
K32(k_fma, F_FMA)
K32(k_mov, F_MOV)
K32(k_cnd, F_CND)
K32(k_addu, F_ADDU)
K32(k_max3, F_MAX3)
K32(k_cmp, F_CMP)
K32(k_sqrt, F_SQRT)
K32(k_rcp, F_RCP)
K32(k_dsc, F_DSC)
K32(k_dfm, F_DFM)
K32(k_dfx, F_DFX)
K32(k_mullo, F_MULLO)
K32(k_mulhi, F_MULHI)
K32(k_dpp, F_DPP)
K32(k_mbcnt, F_MBCNT)
K32(k_bfe, F_BFE)
K64(k_fma64, F_FMA64)
K64(k_mul64, F_MUL64)
K64(k_add64, F_ADD64)
K64(k_lshl64, F_LSHL64)
K64(k_rcp64, F_RCP64)
KPK(k_pkfma, F_PKFMA)
KPK(k_pkmul, F_PKMUL)
KPK(k_pkadd, F_PKADD)
K32(k_fmac, F_FMAC)
K32(k_max, F_MAX)
K32(k_and, F_AND)
K32(k_lshl, F_LSHL)
K32(k_align, F_ALIGN)
K32(k_mule64, F_MULE64)
K32(k_sub, F_SUB)
K32(k_addf, F_ADDF)
K32(k_min, F_MIN)
K32(k_or, F_OR)
K32(k_xor, F_XOR)
K32(k_lshlv, F_LSHLV)
K32(k_mullit, F_MULLIT)
K32(k_med3, F_MED3)

// the compiler's usual select: a compare into VCC (or an SGPR pair) and a v_cndmask reading it,
// four independent (compare, select) pairs per group of eight instructions
#define KCMP(NAME, FMT, ...)                                                                  \
    __global__ void NAME(float* out, float s) {                                                \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;                         \
        for (int i = 0; i < ITERS; i++) {                                                      \
            asm volatile(FMT("%0") FMT("%1") FMT("%2") FMT("%3")                               \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)                              \
                         : "v"(s)                                                              \
                         : __VA_ARGS__);                                                       \
        }                                                                                      \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;                        \
    }
#define F_CMPVCND4(r) "v_cmp_lt_f32 vcc, " r ", %4\n v_cndmask_b32 " r ", " r ", %4, vcc\n"
#define F_CMPSCND4(r) "v_cmp_lt_f32 s[20:21], " r ", %4\n v_cndmask_b32_e64 " r ", " r ", %4, s[20:21]\n"
KCMP(k_cmpvcnd, F_CMPVCND4, "vcc")
KCMP(k_cmpscnd, F_CMPSCND4, "s20", "s21")

// v_cndmask_b32 (VCC form) with VCC written by a compare before the loop
__global__ void k_cndv(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    asm volatile("v_cmp_lt_f32 vcc, %0, %1\n s_nop 7" ::"v"(a0), "v"(s) : "vcc");
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n"
            "v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
            "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
            "v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// one dependent chain of v_mul_f32 (latency)
__global__ void k_muldep(float* out, float s) {
    float a0 = threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
            "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
            "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
            : "+v"(a0)
            : "v"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}

// packed multiply by an SGPR pair (the linear scan's form)
__global__ void k_pkmuls(float* out, float s) {
    v2f a0 = {float(threadIdx.x), 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
        a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned long long sv = ((unsigned long long)__float_as_uint(s) << 32) | __float_as_uint(s);
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_pk_mul_f32 %0, %0, %8\n v_pk_mul_f32 %1, %1, %8\n v_pk_mul_f32 %2, %2, %8\n"
            "v_pk_mul_f32 %3, %3, %8\n v_pk_mul_f32 %4, %4, %8\n v_pk_mul_f32 %5, %5, %8\n"
            "v_pk_mul_f32 %6, %6, %8\n v_pk_mul_f32 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "s"(sv));
    }
    v2f t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
}

// v_cndmask_b32 on a lane mask in an SGPR pair set before the loop (the compiler's usual form)
__global__ void k_cnds(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    const unsigned long long m = __ballot(threadIdx.x & 1);
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n"
            "v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n"
            "v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n"
            "v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(s), "s"(m));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// v_mul_f32 with its second operand from an SGPR (VOP2, scalar source)
__global__ void k_muls(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_mul_f32 %0, %8, %0\n v_mul_f32 %1, %8, %1\n v_mul_f32 %2, %8, %2\n"
            "v_mul_f32 %3, %8, %3\n v_mul_f32 %4, %8, %4\n v_mul_f32 %5, %8, %5\n"
            "v_mul_f32 %6, %8, %6\n v_mul_f32 %7, %8, %7\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "s"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// conversions: independent results from a constant input (no chain through the conversion)
__global__ void k_cvt64(float* out, float s) {
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
    float x = s + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_cvt_f64_f32 %0, %8\n v_cvt_f64_f32 %1, %8\n v_cvt_f64_f32 %2, %8\n"
            "v_cvt_f64_f32 %3, %8\n v_cvt_f64_f32 %4, %8\n v_cvt_f64_f32 %5, %8\n"
            "v_cvt_f64_f32 %6, %8\n v_cvt_f64_f32 %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

// VALU -> SGPR: v_readfirstlane_b32 into eight SGPRs
__global__ void k_rfl(float* out, float s) {
    float x = s + threadIdx.x;
    unsigned r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_readfirstlane_b32 %0, %8\n v_readfirstlane_b32 %1, %8\n"
            "v_readfirstlane_b32 %2, %8\n v_readfirstlane_b32 %3, %8\n"
            "v_readfirstlane_b32 %4, %8\n v_readfirstlane_b32 %5, %8\n"
            "v_readfirstlane_b32 %6, %8\n v_readfirstlane_b32 %7, %8\n"
            : "+s"(r0), "+s"(r1), "+s"(r2), "+s"(r3), "+s"(r4), "+s"(r5), "+s"(r6), "+s"(r7)
            : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7);
}

// SALU: eight independent s_add_u32 chains
__global__ void k_salu(float* out, float s) {
    unsigned r0 = blockIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
             r6 = r0 + 6, r7 = r0 + 7;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 3\n s_add_u32 %2, %2, 3\n"
            "s_add_u32 %3, %3, 3\n s_add_u32 %4, %4, 3\n s_add_u32 %5, %5, 3\n"
            "s_add_u32 %6, %6, 3\n s_add_u32 %7, %7, 3\n"
            : "+s"(r0), "+s"(r1), "+s"(r2), "+s"(r3), "+s"(r4), "+s"(r5), "+s"(r6), "+s"(r7)
            :
            : "scc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7);
}

// VALU and SALU interleaved in one wave's stream (4 + 4 per group of 8)
__global__ void k_mix(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned r0 = blockIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_mul_f32 %0, %0, %8\n s_add_u32 %4, %4, 3\n v_mul_f32 %1, %1, %8\n"
            "s_add_u32 %5, %5, 3\n v_mul_f32 %2, %2, %8\n s_add_u32 %6, %6, 3\n"
            "v_mul_f32 %3, %3, %8\n s_add_u32 %7, %7, 3\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(r0), "+s"(r1), "+s"(r2), "+s"(r3)
            : "v"(s)
            : "scc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + (float)(r0 + r1 + r2 + r3);
}

int main(int argc, char** argv) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * 4096 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K {
        const char* name;
        void (*f)(float*, float);
        const char* cls;
    };
    const K ks[] = {
        {"v_mul_f32", k_mul, "valu32"},          {"v_fma_f32", k_fma, "valu32"},
        {"v_mov_b32", k_mov, "valu32"},          {"v_cndmask_b32", k_cnd, "valu32"},
        {"v_add_u32", k_addu, "valu32"},         {"v_max3_f32", k_max3, "valu32"},
        {"v_cmp_lt_f32", k_cmp, "cmp"},          {"v_sqrt_f32", k_sqrt, "trans"},
        {"v_rcp_f32", k_rcp, "trans"},           {"v_div_scale_f32", k_dsc, "div"},
        {"v_div_fmas_f32", k_dfm, "div"},        {"v_div_fixup_f32", k_dfx, "div"},
        {"v_mul_lo_u32", k_mullo, "mul32"},      {"v_mul_hi_u32", k_mulhi, "mul32"},
        {"v_add_u32_dpp", k_dpp, "dpp"},         {"v_mbcnt_lo_u32_b32", k_mbcnt, "valu32"},
        {"v_bfe_u32", k_bfe, "valu32"},          {"v_fma_f64", k_fma64, "f64"},
        {"v_mul_f64", k_mul64, "f64"},           {"v_add_f64", k_add64, "f64"},
        {"v_lshl_add_u64", k_lshl64, "int64"},   {"v_rcp_f64", k_rcp64, "trans64"},
        {"v_pk_fma_f32", k_pkfma, "packed"},     {"v_pk_mul_f32", k_pkmul, "packed"},
        {"v_pk_add_f32", k_pkadd, "packed"},     {"v_cvt_f64_f32", k_cvt64, "cvt64"},
        {"v_readfirstlane_b32", k_rfl, "lane"},  {"s_add_u32", k_salu, "salu"},
        {"mix_v_mul_s_add", k_mix, "mix"},   {"v_fmac_f32", k_fmac, "valu32"},
        {"v_max_f32", k_max, "valu32"},          {"v_and_b32", k_and, "valu32"},
        {"v_lshlrev_b32", k_lshl, "valu32"},     {"v_alignbit_b32", k_align, "valu32"},
        {"v_mul_f32_e64", k_mule64, "valu32"},   {"v_sub_f32", k_sub, "valu32"},
        {"v_cndmask_b32_e64_sgpr", k_cnds, "valu32"}, {"v_mul_f32_sgpr", k_muls, "valu32"},
        {"v_add_f32", k_addf, "valu32"},         {"v_min_f32", k_min, "valu32"},
        {"v_or_b32", k_or, "valu32"},            {"v_xor_b32", k_xor, "valu32"},
        {"v_lshlrev_b32_v", k_lshlv, "valu32"},  {"v_mul_f32_literal", k_mullit, "valu32"},
        {"v_med3_f32", k_med3, "valu32"},        {"cmp_vcc_cndmask", k_cmpvcnd, "pair"},
        {"cmp_sgpr_cndmask_e64", k_cmpscnd, "pair"}, {"v_cndmask_b32_vcc_set", k_cndv, "valu32"},
        {"v_mul_f32_dependent", k_muldep, "valu32"}, {"v_pk_mul_f32_sgpr", k_pkmuls, "packed"},
    };
    const char* only = argc > 1 ? argv[1] : nullptr;  // one form (for a PMC run), or all
    std::printf("{\"cus\": %d, \"iters\": %d, \"forms\": [\n", cus, ITERS);
    bool first = true;
    for (const K& k : ks) {
        if (only && std::strcmp(only, k.name) != 0) continue;
        double ms_at[3] = {0, 0, 0};
        const int wps[3] = {1, 8, 5};  // waves per SIMD: 256-thread blocks are 4 waves (one/SIMD)
        for (int w = 0; w < 3; w++) {
            const int grid = cus * wps[w];
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 0.999f);
            hipEventRecord(e0);
            const int reps = 5;
            for (int r = 0; r < reps; r++)
                hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 0.999f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms_at[w] = ms / reps;
        }
        // wave-instructions per SIMD of the timed loop: waves per SIMD x ITERS x 8
        std::printf("%s {\"form\": \"%s\", \"class\": \"%s\", \"ms_1wave\": %.5f, "
                    "\"ms_8waves\": %.5f, \"ms_5waves\": %.5f, \"insts_per_simd_1wave\": %d}",
                    first ? " " : ",\n ", k.name, k.cls, ms_at[0], ms_at[1], ms_at[2],
                    ITERS * 8);
        first = false;
    }
    std::printf("\n]}\n");
    return 0;
}

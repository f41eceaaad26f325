// microbench_valu.hip -- issue-rate check of VALU forms on gfx950: v_mul_f32 vs
// v_pk_mul_f32 vs v_fma_f32 (same lane-op count), to decide whether packed math pays, and the
// fp64 mul / add / fma the canonical sin is built from.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

__global__ void k_mul(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n"
            "v_mul_f32 %3, %3, %8\n v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n"
            "v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "s"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_pkmul(float* out, float s) {
    f2 a0 = {float(threadIdx.x), 1}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    f2 sv = {s, s};
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n"
            "v_pk_mul_f32 %3, %3, %4\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
            : "v"(sv));
    }
    f2 t = a0 + a1 + a2 + a3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
}

__global__ void k_fma(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n"
            "v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n"
            "v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "s"(s));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// fp64 forms (the canonical sin runs in double): 8 independent chains of one op each
#define F64_KERNEL(NAME, INSN)                                                               \
    __global__ void NAME(float* out, float s) {                                               \
        double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,         \
               a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, sv = s;                                \
        for (int i = 0; i < ITERS; i++) {                                                     \
            asm volatile(INSN " %0, %0, %8\n " INSN " %1, %1, %8\n " INSN " %2, %2, %8\n "   \
                         INSN " %3, %3, %8\n " INSN " %4, %4, %8\n " INSN " %5, %5, %8\n "   \
                         INSN " %6, %6, %8\n " INSN " %7, %7, %8\n"                          \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),        \
                           "+v"(a6), "+v"(a7)                                                 \
                         : "v"(sv));                                                          \
        }                                                                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7); \
    }
F64_KERNEL(k_mul64, "v_mul_f64")
F64_KERNEL(k_add64, "v_add_f64")

__global__ void k_fma64(float* out, float s) {
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, sv = s;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(
            "v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n"
            "v_fma_f64 %3, %3, %8, %8\n v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n"
            "v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(sv));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int block = 256;
    float* out;
    hipMalloc(&out, sizeof(float) * 4096 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K { const char* name; void (*f)(float*, float); double lane_ops; };
    K ks[] = {{"v_mul_f32", k_mul, 8.0 * ITERS}, {"v_pk_mul_f32", k_pkmul, 8.0 * ITERS},
              {"v_fma_f32", k_fma, 8.0 * ITERS}, {"v_mul_f64", k_mul64, 8.0 * ITERS},
              {"v_add_f64", k_add64, 8.0 * ITERS}, {"v_fma_f64", k_fma64, 8.0 * ITERS}};
    for (int wpc : {4, 8, 16, 32}) {
        const int grid = cus * wpc / 4;
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 0.999f);
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++)
                hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 0.999f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops = k.lane_ops * grid * block * 5;  // fp32 lane-ops (mul or fma)
            std::printf("waves/CU %2d %-13s %.2f Tlane-op/s\n", wpc, k.name, ops / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}

// Where do the tracer's f64 accumulation atomics execute? Each kernel adds 1.0 to 4 M doubles
// (32 MB), 4 adds per address from one wave (the tracer's pattern: a pixel's chunks all come
// from one wave), with agent-scope atomics (HIP atomicAdd), workgroup-scope atomics, and plain
// load-add-store. Run under rocprofv3 --pmc WRITE_SIZE (and FETCH_SIZE) to see which of them
// reach the memory side (TCC_EA writes) and which stay in the XCD's L2.
//   hipcc --offload-arch=gfx950 -O3 tools/atomic_scope_probe.hip -o tools/atomic_scope_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 1 << 22;  // doubles
constexpr int kRep = 4;

__global__ void add_agent(double* a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < kRep; r++) atomicAdd(a + i, 1.0);
}

__global__ void add_workgroup(double* a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < kRep; r++)
        __hip_atomic_fetch_add(a + i, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ void add_wavefront(double* a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < kRep; r++)
        __hip_atomic_fetch_add(a + i, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__global__ void add_plain(double* a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < kRep; r++) {
        volatile double* v = a + i;
        *v = *v + 1.0;
    }
}

int main() {
    double* a = nullptr;
    if (hipMalloc(&a, sizeof(double) * kN) != hipSuccess) return 1;
    int bad = 0;
    void (*ks[4])(double*) = {add_agent, add_workgroup, add_wavefront, add_plain};
    const char* names[4] = {"agent", "workgroup", "wavefront", "plain"};
    for (int k = 0; k < 4; k++) {
        (void)hipMemset(a, 0, sizeof(double) * kN);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(ks[k], dim3(kN / 256), dim3(256), 0, 0, a);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        double h[4];
        (void)hipMemcpy(h, a + 12345, sizeof(h), hipMemcpyDeviceToHost);
        const bool ok = h[0] == kRep && h[3] == kRep;
        bad += !ok;
        std::printf("%-10s %.3f ms  value %.1f %s\n", names[k], ms, h[0], ok ? "ok" : "WRONG");
    }
    (void)hipFree(a);
    return bad;
}

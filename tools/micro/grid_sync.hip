// Cost of a grid-wide barrier on MI355X: cooperative_groups grid.sync() against a counter barrier with
// agent-scope fences, N barriers in one cooperative launch (every workgroup resident).
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <cstdio>
namespace cg = cooperative_groups;

__global__ void k_cg(unsigned* x, int n) {
    cg::grid_group g = cg::this_grid();
    for (int i = 0; i < n; ++i) {
        if (threadIdx.x == 0) atomicAdd(x + (i & 1), 1u);
        g.sync();
    }
}

__device__ __forceinline__ void bar(unsigned* c, unsigned target) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++spins < (1u << 24))
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__global__ void k_ctr(unsigned* x, unsigned* c, int n) {
    for (int i = 0; i < n; ++i) {
        if (threadIdx.x == 0) atomicAdd(x + (i & 1), 1u);
        bar(c, (unsigned)(i + 1) * gridDim.x);
    }
}

int main() {
    unsigned *x, *c;
    (void)hipMalloc(&x, 8);
    (void)hipMalloc(&c, 4);
    int cus = 0, nb = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_cg, 256, 0);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int per : {1, 2, 4}) {
        for (int which = 0; which < 2; ++which) {
            int n = 2000;
            dim3 grid(per * cus);
            (void)hipMemset(c, 0, 4);
            void* args_cg[] = {&x, &n};
            void* args_ctr[] = {&x, &c, &n};
            (void)hipEventRecord(a);
            hipError_t e = which == 0 ? hipLaunchCooperativeKernel((const void*)k_cg, grid, dim3(256), args_cg, 0, 0)
                                      : hipLaunchCooperativeKernel((const void*)k_ctr, grid, dim3(256), args_ctr, 0, 0);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("%s blocks=%d (occupancy %d per CU): %s, %.2f us per barrier\n", which ? "counter" : "cg", per * cus,
                   nb, hipGetErrorString(e), ms * 1000 / n);
        }
    }
    return 0;
}

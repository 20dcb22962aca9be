// LDS residency probe: how many 64-thread workgroups with a given dynamic LDS size run at once
// on one CU of this GPU (the allocation granularity decides it).  Every workgroup
// records the realtime clock at start, sleeps ~2 ms, and stops; workgroups that started within
// 0.5 ms of the first one were resident in the first round.  Bounded: no workgroup waits on another.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

extern "C" __global__ __launch_bounds__(64) void probe(unsigned long long *t) {
    extern __shared__ unsigned int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) __builtin_amdgcn_s_sleep(64);  // 2 ms at 100 MHz
    if (threadIdx.x == 0) t[blockIdx.x] = t0 + lds[1];
}

int main(int argc, char **argv) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 1;
    const int n_cu = p.multiProcessorCount;
    printf("{\"cus\": %d, \"lds_per_cu\": %zu, \"results\": [", n_cu, (size_t)p.maxSharedMemoryPerMultiProcessor);
    const int sizes[] = {7680, 8192, 9216, 9504, 9728, 9984, 10240, 10368, 10752, 11264, 11376, 13264, 17056, 20752, 24496, 32016, 39504, 50768, 62000};
    bool first = true;
    for (int sz : sizes) {
        const int n = n_cu * 48;
        unsigned long long *d = nullptr;
        if (hipMalloc(&d, 8 * (size_t)n) != hipSuccess) return 1;
        if (sz > 65536) (void)hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, sz);
        hipLaunchKernelGGL(probe, dim3(n), dim3(64), sz, 0, d);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        std::vector<unsigned long long> h(n);
        (void)hipMemcpy(h.data(), d, 8 * (size_t)n, hipMemcpyDeviceToHost);
        (void)hipFree(d);
        const unsigned long long t0 = *std::min_element(h.begin(), h.end());
        int round1 = 0;
        for (auto v : h) round1 += (v - t0) < 50000ull;  // within 0.5 ms
        printf("%s{\"lds\": %d, \"resident\": %d, \"per_cu\": %.3f}", first ? "" : ", ", sz, round1, (double)round1 / n_cu);
        first = false;
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}

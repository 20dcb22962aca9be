// checks the DPP wave scans / lane moves of mt_snapshot.hip against a host computation (one wave)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
__device__ __forceinline__ unsigned incl(unsigned v) {
    unsigned x = v;
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
__global__ void k(const unsigned *in, unsigned *o) {
    const unsigned t = threadIdx.x, v = in[t];
    o[t] = incl(v);
    o[64 + t] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
    o[128 + t] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}
int main() {
    unsigned h[64], r[192], *di, *dout;
    srand(7);
    int bad = 0;
    hipMalloc(&di, sizeof h);
    hipMalloc(&dout, sizeof r);
    for (int it = 0; it < 100; it++) {
        for (int i = 0; i < 64; i++) h[i] = (unsigned)(rand() % 1000);
        hipMemcpy(di, h, sizeof h, hipMemcpyHostToDevice);
        k<<<1, 64>>>(di, dout);
        hipMemcpy(r, dout, sizeof r, hipMemcpyDeviceToHost);
        unsigned s = 0;
        for (int i = 0; i < 64; i++) {
            s += h[i];
            if (r[i] != s) bad++;
            if (r[64 + i] != (i ? h[i - 1] : 0u)) bad++;
            if (r[128 + i] != (i < 63 ? h[i + 1] : 0u)) bad++;
        }
        if (it == 0 && bad) for (int i = 0; i < 64; i++) printf("%d: in %u scan %u prev %u next %u\n", i, h[i], r[i], r[64+i], r[128+i]);
    }
    printf("dpp_scan mismatches: %d\n", bad);
    return bad != 0;
}

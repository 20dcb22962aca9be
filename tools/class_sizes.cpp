// Capacity classes (mt_device.h kClassSegs): for n documents per CU, the largest slot count whose
// LDS layout (make_layout) fits floor(128 / n) granules of 1,280 B.
// build: hipcc -std=c++17 --offload-arch=gfx950 tools/class_sizes.cpp -o /tmp/class_sizes
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../fluidframework_amd/csrc/mt_device.h"
int main() {
    int tiers[] = {16, 14, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1};
    for (int n : tiers) {
        const unsigned budget = (128 / n) * 1280;
        int best = 0;
        for (int seg = 16; seg < 20000; seg++) if (mt::make_layout(seg).bytes <= budget) best = seg;
        printf("%d/CU: seg %d bytes %u (budget %u)\n", n, best, mt::make_layout(best).bytes, budget);
    }

}

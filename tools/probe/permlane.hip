// Probe: semantics of __builtin_amdgcn_permlane{16,32}_swap on gfx950 (which operand's lanes move).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *out) {
    const unsigned l = threadIdx.x;
    const unsigned a = l, b = 100 + l;
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    const auto q = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[l] = r[0]; out[64 + l] = r[1]; out[128 + l] = q[0]; out[192 + l] = q[1];
}
int main() {
    unsigned *d, h[256];
    hipMalloc(&d, 1024);
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    const char *nm[4] = {"p32 r0", "p32 r1", "p16 r0", "p16 r1"};
    for (int v = 0; v < 4; v++) {
        printf("%s:", nm[v]);
        for (int row = 0; row < 4; row++) printf(" [row%d: %u..%u]", row, h[64 * v + 16 * row], h[64 * v + 16 * row + 15]);
        printf("\n");
    }
    return 0;
}

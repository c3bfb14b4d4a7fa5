// Runs g2048_wgrad on exact small-integer data and prints the error pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../include/g2048_ppo.h"
static uint16_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 64, n1 = argc > 2 ? atoi(argv[2]) : 16, n2 = argc > 3 ? atoi(argv[3]) : 16;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    std::vector<uint16_t> a(m * n1), b(m * n2);
    std::vector<double> ref(n1 * n2, 0.0);
    for (int r = 0; r < m; r++) {
        for (int i = 0; i < n1; i++) a[r * n1 + i] = bf(mode == 0 ? (r == i ? 1.0f : 0.0f) : (float)((r * 7 + i * 3) % 5 - 2));
        for (int j = 0; j < n2; j++) b[r * n2 + j] = bf(mode == 0 ? (float)(16 * (r % 16) + j) : (float)((r * 5 + j * 11) % 7 - 3));
    }
    for (int r = 0; r < m; r++)
        for (int i = 0; i < n1; i++)
            for (int j = 0; j < n2; j++) {
                float x, y;
                uint32_t ux = (uint32_t)a[r * n1 + i] << 16, uy = (uint32_t)b[r * n2 + j] << 16;
                memcpy(&x, &ux, 4);
                memcpy(&y, &uy, 4);
                ref[i * n2 + j] += (double)x * y;
            }
    uint16_t *da, *db;
    float *dp, *dout;
    size_t np = g2048_wgrad_partials(m, n1, n2);
    (void)hipMalloc(&da, a.size() * 2);
    (void)hipMalloc(&db, b.size() * 2);
    (void)hipMalloc(&dp, np * 4);
    (void)hipMalloc(&dout, n1 * n2 * 4);
    (void)hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b.data(), b.size() * 2, hipMemcpyHostToDevice);
    int st = g2048_wgrad(nullptr, da, db, m, n1, n2, dp, dout);
    std::vector<float> out(n1 * n2);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n1; i++)
        for (int j = 0; j < n2; j++)
            if (out[i * n2 + j] != (float)ref[i * n2 + j]) {
                if (bad < 20) printf("  [%d][%d] got %g want %g\n", i, j, out[i * n2 + j], ref[i * n2 + j]);
                bad++;
            }
    printf("m=%d n1=%d n2=%d mode=%d status=%d bad=%d / %d\n", m, n1, n2, mode, st, bad, n1 * n2);
    return 0;
}

// Times g2048_muon_step on one r x c matrix for ns_steps = 0, 1, 5 (GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/g2048_ppo.h"
int main(int argc, char **argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 196, C = argc > 2 ? atoi(argv[2]) : 196;
    const int n = R * C;
    std::vector<float> h(n);
    for (int i = 0; i < n; i++) h[i] = (float)((i * 7919) % 1000) / 1000.0f - 0.5f;
    float *p, *g, *mom, *lr;
    (void)hipMalloc(&p, n * 4);
    (void)hipMalloc(&g, n * 4);
    (void)hipMalloc(&mom, n * 4);
    (void)hipMalloc(&lr, 16);
    (void)hipMemcpy(g, h.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemset(p, 0, n * 4);
    (void)hipMemset(mom, 0, n * 4);
    float lrs[4] = {1e-3f, 1e-3f, 1e-3f, 1e-3f};
    (void)hipMemcpy(lr, lrs, 16, hipMemcpyHostToDevice);
    g2048_muon_matrix m{p, g, mom, nullptr, R, C, 0, 0};
    for (int steps : {0, 1, 5}) {
        g2048_muon_cfg cfg{0.95f, 0.01f, 3.4445f, -4.775f, 2.0315f, 1e-7f, steps, 1};
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        int st = g2048_muon_step(nullptr, &m, 1, lr, nullptr, &cfg);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, nullptr);
        for (int i = 0; i < 20; i++) st |= g2048_muon_step(nullptr, &m, 1, lr, nullptr, &cfg);
        (void)hipEventRecord(e1, nullptr);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("R=%d C=%d ns_steps=%d status=%d: %.1f us per step\n", R, C, steps, st, ms * 1000 / 20);
    }
    return 0;
}

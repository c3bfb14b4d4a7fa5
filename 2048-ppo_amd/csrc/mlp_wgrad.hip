// mlp_wgrad.hip -- the four weight gradients of the GameMLP minibatch backward (loss.backward(),
// train.py:548-556; the Linear weights of GameMLP, game.py:1145-1220) in ONE launch:
//
//   head   dz^T H2   dz as two bf16 terms [m][16] (hi rows 0-4, lo rows 8-12), H2 = block 2's output
//   stem   dG0^T x0  x0 = the bf16 observations [m][48]
//   block1 dG1^T H0
//   block2 dG2^T H1
//
// replacing three g2048_wgrad launches (head, stem) / g2048_wgrad_pair (blocks): those were
// latency-bound (one 64-row step of loads in flight per CU, 1.4-3.8 TB/s).  Here every CU streams
// one product's contiguous row range with kStages - 1 = 3 stages of 32 rows in flight through
// LDS-DMA (buffer_load ... lds: no registers, a counted vmcnt and a raw s_barrier per stage,
// cdna_hip_programming.md §5 "Pipelining across barriers").  The CUs are shared out among the
// products in proportion to their bytes per row, so all four finish together; each block writes one
// fp32 partial of its product, summed in a fixed order by g2048_colsum_batch (deterministic).
//
// Stage layout: per operand a 16 KiB region holding the 32 rows exactly as they lie in HBM (lane-
// linear LDS-DMA: 1 KiB per wave-instruction); chunks past the stage's rows are sent out of the
// buffer range (zeros), so every wave issues the same instruction count (the counted waits hold).
// The MFMA operands (v_mfma_f32_16x16x32_bf16, K = rows) come from the unpadded row-major image by
// the transposing ds_read_b64_tr_b16 (the g2048_wgrad fragment pattern).  Rows past the block's
// range read as zero in both operands (buffer range check), so a ragged m needs no other masking;
// output tiles past n1 / n2 read neighbouring bytes and are dropped at the store.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/g2048_ppo.h"

#include "wgrad_ring.hpp"

using namespace g2048::wgr;

namespace {

enum { kHead = 0, kStem = 1, kBlock1 = 2, kBlock2 = 3, kProducts = 4 };


struct Args {
    Prod p[kProducts];
    int64_t m;
};

template <int H>
__global__ __launch_bounds__(kThreads) void mlp_wgrad_kernel(Args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int b = blockIdx.x;
    // block -> product (block-uniform)
    int k = kProducts - 1;
    while (k > 0 && b < a.p[k].blk0) k--;
    const int blk = b - a.p[k].blk0;
    if (blk >= a.p[k].nb) return;
    constexpr int TH = (H + 15) / 16;
    switch (k) {
    case kHead: product<16, H, 1, (TH + 7) / 8, 1>(a.p[k], a.m, blk, smem); break;
    case kStem: product<H, 48, (TH + 7) / 8, 3, 8>(a.p[k], a.m, blk, smem); break;
    default: product<H, H, (TH + 1) / 2, (TH + 3) / 4, 2>(a.p[k], a.m, blk, smem); break;
    }
}

inline bool al16(const void *p) { return ((uintptr_t)p % 16) == 0u; }

// blocks per product in proportion to its bytes per row (head 32 + 2h, stem 2h + 96, blocks 4h each)
struct Plan {
    int nb[kProducts];
    int64_t rows[kProducts];
    int total;
};

Plan plan(int64_t m, int h) {
    Plan p{};
    const double w[kProducts] = {32.0 + 2.0 * h, 2.0 * h + 96.0, 4.0 * h, 4.0 * h};
    const double W = w[0] + w[1] + w[2] + w[3];
    const int64_t max_nb = (m + kRows - 1) / kRows;
    p.total = 0;
    for (int k = 0; k < kProducts; k++) {
        int64_t nb = (int64_t)(kMaxBlocks * w[k] / W);
        nb = nb < 1 ? 1 : (nb > max_nb ? max_nb : nb);
        int64_t rows = (m + nb - 1) / nb;
        rows = (rows + kRows - 1) / kRows * kRows;
        p.rows[k] = rows;
        p.nb[k] = (int)((m + rows - 1) / rows);
        p.total += p.nb[k];
    }
    return p;
}

bool shape_ok(int h) { return h == 196 || h == 192 || h == 128 || h == 64 || h == 32; }

}  // namespace

extern "C" {

size_t g2048_mlp_wgrad_partials(int64_t m, int32_t hidden) {
    if (m <= 0 || !shape_ok(hidden)) return 0;
    const Plan p = plan(m, hidden);
    const size_t h = (size_t)hidden;
    return (size_t)p.nb[kHead] * 16 * h + (size_t)p.nb[kStem] * h * 48 + (size_t)(p.nb[kBlock1] + p.nb[kBlock2]) * h * h;
}

int g2048_mlp_wgrad(g2048_stream_t stream, const g2048_mlp_wgrad_args *args, float *out_head, float *const *out_w,
                    g2048_colsum_job *defer) {
    if (!args || !out_head || !out_w || !out_w[0] || !out_w[1] || !out_w[2]) return G2048_EINVAL;
    const int h = args->hidden;
    const int64_t m = args->m;
    if (m <= 0 || !shape_ok(h) || !args->partials || m * 4 * h >= (int64_t(1) << 31)) return G2048_EINVAL;
    const void *ops[8] = {args->dz_bf16, args->h2, args->dg[0], args->x[0], args->dg[1], args->x[1], args->dg[2], args->x[2]};
    for (const void *q : ops)
        if (!q || !al16(q)) return G2048_EINVAL;
    const Plan pl = plan(m, h);
    Args a{};
    a.m = m;
    const int n1[kProducts] = {16, h, h, h}, n2[kProducts] = {h, 48, h, h};
    float *part = args->partials;
    int blk0 = 0;
    for (int k = 0; k < kProducts; k++) {
        a.p[k].a = static_cast<const char *>(ops[2 * k]);
        a.p[k].b = static_cast<const char *>(ops[2 * k + 1]);
        a.p[k].part = part;
        a.p[k].rows = pl.rows[k];
        a.p[k].nb = pl.nb[k];
        a.p[k].blk0 = blk0;
        part += (size_t)pl.nb[k] * n1[k] * n2[k];
        blk0 += pl.nb[k];
    }
    const hipStream_t s = (hipStream_t)stream;
    switch (h) {
    case 196: hipLaunchKernelGGL(mlp_wgrad_kernel<196>, dim3(pl.total), dim3(kThreads), kLds, s, a); break;
    case 192: hipLaunchKernelGGL(mlp_wgrad_kernel<192>, dim3(pl.total), dim3(kThreads), kLds, s, a); break;
    case 128: hipLaunchKernelGGL(mlp_wgrad_kernel<128>, dim3(pl.total), dim3(kThreads), kLds, s, a); break;
    case 64: hipLaunchKernelGGL(mlp_wgrad_kernel<64>, dim3(pl.total), dim3(kThreads), kLds, s, a); break;
    default: hipLaunchKernelGGL(mlp_wgrad_kernel<32>, dim3(pl.total), dim3(kThreads), kLds, s, a); break;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    g2048_colsum_job jobs[kProducts];
    float *dst[kProducts] = {out_head, out_w[0], out_w[1], out_w[2]};
    for (int k = 0; k < kProducts; k++) {
        jobs[k] = g2048_colsum_job{};
        jobs[k].part = a.p[k].part;
        jobs[k].nb = pl.nb[k];
        jobs[k].cols = n1[k] * n2[k];
        jobs[k].max_col = -1;
        jobs[k].nseg = 1;
        jobs[k].dst[0] = dst[k];
        jobs[k].len[0] = n1[k] * n2[k];
    }
    if (defer) {
        for (int k = 0; k < kProducts; k++) defer[k] = jobs[k];
        return G2048_OK;
    }
    return g2048_colsum_batch(stream, jobs, kProducts);
}

}  // extern "C"

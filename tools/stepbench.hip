// stepbench.hip -- development tool: shader-clock cost of one candidate step
// (eval_candidates + selection) of the macroblock search, per partition
// shape, on synthetic planes.  One 512-lane workgroup, MB (1, 1) of a
// 64x64 picture.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/stepbench tools/stepbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../hartallo_amd/csrc/hl_mbcore.h"

using namespace hl;

constexpr int kIters = 200;

__global__ __launch_bounds__(kMbThreads) void k_step(FrameArgs F, long long* out)
{
    __shared__ Shared S;
    const int tid = threadIdx.x;
    Ctx c{F, S, tid, kMbThreads, 5, 1, 1, 16, 16, 9, 0, 0, S.lk[tid & 15]};
    if (tid < 16) S.lk[tid] = make_lanek(tid, F.qp, F.qpc);
    c.Q = make_laneq(tid, F.qp);
    __syncthreads();
    mb_begin(c);
    static constexpr int shapes[7][2] = {{16, 16}, {16, 8}, {8, 16}, {8, 8}, {8, 4}, {4, 8}, {4, 4}};
    for (int sh = 0; sh < 7; ++sh)
        for (int nc = 1; nc <= 9; nc += 8) {
            PartGeo g;
            g.px = g.py = 0;
            g.pw = shapes[sh][0];
            g.ph = shapes[sh][1];
            g.nbw = g.pw >> 2;
            g.nblk = (g.pw >> 2) * (g.ph >> 2);
            g.lbw = ilog2_small(g.nbw);
            g.lnb = ilog2_small(g.nblk);
            const int pmv[2] = {2, -1};
            HL_SYNC();
#if defined(HL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
            for (int i = 0; i < kProfSlots; ++i) c.pacc[i] = 0;
#endif
            const long long t0 = __builtin_readcyclecounter();
            int acc = 0;
            for (int it = 0; it < kIters; ++it) {
                for (int i = 0; i < nc; ++i) put_cand(c, g.px, g.py, i, ((it + i) % 7) - 3, ((it * 3 + i) % 5) - 2, i, (tid & 63) == 0);
                eval_candidates(c, g, nc, pmv);
                double m;
                acc += pick_first_min(c, 0, nc, m);
            }
            const long long t1 = __builtin_readcyclecounter();
            if (tid == 0) {
                out[8 * (sh * 2 + (nc > 1))] = (t1 - t0) / kIters;
                out[8 * (sh * 2 + (nc > 1)) + 1] = acc;
#if defined(HL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
                for (int i = 0; i < 7; ++i) out[8 * (sh * 2 + (nc > 1)) + 1 + i] = c.pacc[i] / kIters;
#endif
            }
        }
}

int main()
{
    const int W = 64, H = 64, mbw = 4, mbh = 4;
    FrameArgs F{};
    F.W = W;
    F.H = H;
    F.Wc = W / 2;
    F.Hc = H / 2;
    F.mbw = mbw;
    F.mbh = mbh;
    F.qp = 28;
    F.qpc = kQpToQpc[28];
    F.me_range = 16;
    F.lambda = 0.852 * (double)(1 << ((28 - 12) / 3));
    const int pstride = (W + 2 * kPad + 63) & ~63, pls = pstride * (H + 2 * kPad);
    uint8_t *src, *cur, *ref, *pl;
    hipMalloc(&src, W * H * 3 / 2);
    hipMalloc(&cur, W * H * 3 / 2);
    hipMalloc(&ref, W * H * 3 / 2);
    hipMalloc(&pl, 4 * pls);
    uint8_t* h = (uint8_t*)malloc(4 * pls);
    srand(1);
    for (int i = 0; i < 4 * pls; ++i) h[i] = (uint8_t)(128 + (rand() % 40) - 20);
    hipMemcpy(pl, h, 4 * pls, hipMemcpyHostToDevice);
    hipMemcpy(src, h + 5000, W * H * 3 / 2, hipMemcpyHostToDevice);
    hipMemcpy(cur, h + 9000, W * H * 3 / 2, hipMemcpyHostToDevice);
    hipMemcpy(ref, h + 13000, W * H * 3 / 2, hipMemcpyHostToDevice);
    F.src[0] = src;
    F.src[1] = src + W * H;
    F.src[2] = src + W * H * 5 / 4;
    F.cur[0] = cur;
    F.cur[1] = cur + W * H;
    F.cur[2] = cur + W * H * 5 / 4;
    F.ref[0] = ref;
    F.ref[1] = ref + W * H;
    F.ref[2] = ref + W * H * 5 / 4;
    for (int i = 0; i < 4; ++i) F.pl[i] = pl + i * pls;
    F.pstride = pstride;
    F.plsz = pls;
    MbState* st;
    hipMalloc(&st, sizeof(MbState) * mbw * mbh);
    hipMemset(st, 0, sizeof(MbState) * mbw * mbh);
    F.st = st;
    long long* out;
    hipMalloc(&out, 128 * sizeof(long long));
    for (int r = 0; r < 2; ++r) k_step<<<1, kMbThreads>>>(F, out);
    long long o[128];
    hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
    const char* names[7] = {"16x16", "16x8", "8x16", "8x8", "8x4", "4x8", "4x4"};
    for (int sh = 0; sh < 7; ++sh)
        for (int k = 0; k < 2; ++k) {
            const long long* r = o + 8 * (sh * 2 + k);
            printf("%-6s %d cand: step %6lld  [A %5lld  B %5lld  tail %5lld | A: slot+load %5lld  fwd+q %5lld  cavlc %5lld  idct+dist %5lld]\n",
                   names[sh], k ? 9 : 1, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
        }
    return 0;
}

// cavlcbench.hip -- development tool: cycles of the cooperative 4x4 pieces in
// isolation (one 512-lane workgroup, 32 rows).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../hartallo_amd/csrc/hl_coop.h"

using namespace hl;

__global__ __launch_bounds__(512) void k_cb(const int* in, int* out, long long* cyc)
{
    __shared__ CoopTables T;
    __shared__ alignas(16) int lvs[32][16];
    coop_tables_init(T, threadIdx.x, 512);
    __syncthreads();
    const LaneK K = make_lanek(threadIdx.x, 28, 28);
    int q = in[threadIdx.x];
    int acc = 0;
    long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < 100; ++i) {
        const CoopStat st = coop_cavlc(T, q, K.s, lvs[threadIdx.x >> 4]);
        acc += st.rest + st.tc;
        q ^= (acc & 1);
    }
    long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[0] = (t1 - t0) / 100;
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < 100; ++i) {
        acc += coop_fwd(K, q + acc);
    }
    t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[1] = (t1 - t0) / 100;
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < 100; ++i) {
        acc += coop_idct(K, coop_dequant(q + (acc & 3), K.ls, 28));
    }
    t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[2] = (t1 - t0) / 100;
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < 100; ++i) acc += row_sum(acc);
    t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[3] = (t1 - t0) / 100;
    out[threadIdx.x] = acc;
}

int main()
{
    int h[512];
    for (int i = 0; i < 512; ++i) h[i] = (i * 7919 % 13) - 6 > 3 ? ((i * 31) % 5) - 2 : 0;
    int *in, *out;
    long long* cyc;
    (void)hipMalloc(&in, sizeof(h));
    (void)hipMalloc(&out, sizeof(h));
    (void)hipMalloc(&cyc, 64);
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 3; ++r) k_cb<<<1, 512>>>(in, out, cyc);
    long long c[4];
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("coop_cavlc %lld  coop_fwd %lld  dequant+idct %lld  row_sum %lld cycles\n", c[0], c[1], c[2], c[3]);
    return 0;
}

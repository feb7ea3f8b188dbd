// microbench.hip -- development tool: shader-clock cost of the primitives the
// macroblock step is built from, on one 512-lane workgroup (8 waves).
//   hipcc --offload-arch=gfx950 -O3 -o build/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 256

__global__ __launch_bounds__(512) void k_bench(const int* g, int* out, long long* cyc)
{
    __shared__ int lds[4096];
    const int tid = threadIdx.x;
    for (int i = tid; i < 4096; i += 512) lds[i] = i;
    __syncthreads();
    long long t0, t1;
    int acc = tid;
    // 1. barrier only
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) __syncthreads();
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[0] = (t1 - t0) / N;
    // 2. dependent LDS read chain (one wave's lanes)
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) acc = lds[(acc + i) & 4095];
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[1] = (t1 - t0) / N;
    // 3. LDS write by one lane, barrier, read by all
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) {
        if (tid == 0) lds[i] = acc;
        __syncthreads();
        acc += lds[i];
    }
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[2] = (t1 - t0) / N;
    // 4. dependent DPP row_ror chain
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) acc += __builtin_amdgcn_update_dpp(0, acc, 0x124, 0xF, 0xF, false);
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[3] = (t1 - t0) / N;
    // 5. dependent VALU add chain
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) acc = acc * 3 + i;
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[4] = (t1 - t0) / N;
    // 6. dependent global load chain (L2-resident 1 MB)
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) acc = g[(acc * 4099 + i * 64) & ((1 << 18) - 1)] & 0xFFFF;
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[5] = (t1 - t0) / N;
    // 7. readcyclecounter back-to-back
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) acc += (int)__builtin_readcyclecounter();
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[6] = (t1 - t0) / N;
    // 8. ballot + readfirstlane chain
    t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) acc += __builtin_amdgcn_readfirstlane((int)__ballot(acc & 1));
    t1 = __builtin_readcyclecounter();
    if (tid == 0) cyc[7] = (t1 - t0) / N;
    out[tid] = acc;
}

int main()
{
    int *g, *out;
    long long* cyc;
    hipMalloc(&g, 4 << 20);
    hipMemset(g, 1, 4 << 20);
    hipMalloc(&out, 512 * 4);
    hipMalloc(&cyc, 8 * 8);
    for (int r = 0; r < 3; ++r) k_bench<<<1, 512>>>(g, out, cyc);
    long long h[8];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[8] = {"barrier (8 waves)", "dependent LDS read", "lane0 LDS write+barrier+read", "dependent DPP row_ror+add",
                            "dependent v_mad chain", "dependent global load (L2)", "readcyclecounter", "ballot+readfirstlane+add"};
    for (int i = 0; i < 8; ++i) printf("%-32s %6lld cycles\n", names[i], h[i]);
    return 0;
}

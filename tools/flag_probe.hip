// Development probe: when does a host poller see a flag that a running
// kernel stores into pinned host memory?  One workgroup spins ~200 ms and
// stores 1, 2, 3 at ~50 ms intervals with a system-scope release store;
// the host prints the time it first sees each value, for several pinned
// allocation flavours.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>
#include <thread>

__global__ void k_flag(int* flag, long long cycles_per_step)
{
    if (threadIdx.x != 0) return;
    for (int v = 1; v <= 3; ++v) {
        const long long t0 = clock64();
        while (clock64() - t0 < cycles_per_step) {}
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static void run(const char* name, int* host, int* dev)
{
    __atomic_store_n(host, 0, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, 0, dev, 100000000LL);  // ~ 50 ms per step at ~2 GHz
    int seen = 0;
    double at[4] = {0, 0, 0, 0};
    while (seen < 3) {
        const int v = __atomic_load_n(host, __ATOMIC_ACQUIRE);
        const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (v > seen) {
            for (int k = seen + 1; k <= v; ++k) at[k] = t;
            seen = v;
        }
        if (t > 5000) break;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    (void)hipDeviceSynchronize();
    const double end = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("%-28s seen 1 at %7.2f ms, 2 at %7.2f, 3 at %7.2f, kernel done by %7.2f\n", name, at[1], at[2], at[3], end);
}

int main()
{
    struct { const char* name; unsigned flags; } kinds[] = {
        {"hipHostMallocDefault", hipHostMallocDefault},
        {"Mapped|Coherent", hipHostMallocMapped | hipHostMallocCoherent},
        {"Coherent", hipHostMallocCoherent},
        {"Mapped|NonCoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
    };
    for (auto& k : kinds) {
        int* h = nullptr;
        int* d = nullptr;
        if (hipHostMalloc((void**)&h, 64, k.flags) != hipSuccess || hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) {
            printf("%s: allocation failed\n", k.name);
            continue;
        }
        run(k.name, h, d);
        (void)hipHostFree(h);
    }
    return 0;
}

// launch_cost.hip -- host time of one kernel launch by kernel-argument size
// (the drop-in miss launches k_add1_row with ~400 B of arguments): an empty
// kernel taking 16 B, 128 B, 256 B or 448 B of arguments, launched N times
// back to back (no waiting inside the timed loop), then the same through
// hipModuleLaunchKernel-style hipLaunchKernel with a cached function pointer.
// Prints one JSON line.  hipcc --offload-arch=gfx950 -O2 launch_cost.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int W>
struct Args {
    unsigned int w[W];
};

template <int W>
__global__ void k_empty(Args<W> a) {
    if (a.w[0] == 0xFFFFFFFFu && threadIdx.x == 0) a.w[1] = 0;   // never true; keeps the argument live
}

template <int W>
double launch_us(hipStream_t s, int n, int grid) {
    Args<W> a{};
    a.w[0] = 1;
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_empty<W>, dim3(grid), dim3(128), 0, s, a);
    hipStreamSynchronize(s);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) {
        a.w[W - 1] = i;
        hipLaunchKernelGGL(k_empty<W>, dim3(grid), dim3(128), 0, s, a);
        if ((i & 63) == 63) hipStreamSynchronize(s);   // keep the queue short, as the miss path does
    }
    hipStreamSynchronize(s);
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
}

// one launch and a spin on a pinned flag the kernel writes (the miss path's shape)
__global__ void k_flag(volatile unsigned int *f, unsigned int v, Args<100> a) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.w[0] != 0xFFFFFFFFu) {
        __threadfence_system();
        *f = v;
    }
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int n = 4000;
    double r16 = launch_us<4>(s, n, 256), r128 = launch_us<32>(s, n, 256), r256 = launch_us<64>(s, n, 256),
           r448 = launch_us<112>(s, n, 256);
    double g1 = launch_us<112>(s, n, 1);
    unsigned int *f = nullptr;
    hipHostMalloc((void **)&f, 64, hipHostMallocMapped);
    unsigned int *fd = nullptr;
    hipHostGetDevicePointer((void **)&fd, f, 0);
    *f = 0;
    Args<100> a{};
    a.w[0] = 1;
    double tot = 0, launch = 0;
    for (int i = 1; i <= 2000; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_flag, dim3(256), dim3(128), 0, s, fd, (unsigned)i, a);
        const auto t1 = std::chrono::steady_clock::now();
        while (*(volatile unsigned int *)f != (unsigned)i) {
        }
        const auto t2 = std::chrono::steady_clock::now();
        tot += std::chrono::duration<double, std::micro>(t2 - t0).count();
        launch += std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    hipStreamSynchronize(s);
    printf("{\"launch_us_args16\": %.3f, \"launch_us_args128\": %.3f, \"launch_us_args256\": %.3f, "
           "\"launch_us_args448\": %.3f, \"launch_us_args448_grid1\": %.3f, \"flag_roundtrip_us\": %.3f, "
           "\"flag_launch_us\": %.3f}\n",
           r16, r128, r256, r448, g1, tot / 2000, launch / 2000);
    hipHostFree(f);
    hipStreamDestroy(s);
    return 0;
}

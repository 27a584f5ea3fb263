// Round-trip latency of the ways a host thread can wait for one small launch
// on MI355X (input to the per-pair ForklessCause miss path):
//   stream_sync   launch + hipStreamSynchronize
//   event_sync    launch + hipEventRecord + hipEventSynchronize
//   spin_flag     launch whose last workgroup stores a sequence number into
//                 pinned host memory (system-scope release), host spins on it
//   two_kernels   two dependent launches + hipStreamSynchronize
//   write_value   launch + hipStreamWriteValue32 into pinned memory, host spins
// hipcc --offload-arch=gfx950 -O2 -o sync_latency sync_latency.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(uint32_t *d) { if (threadIdx.x == 0 && blockIdx.x == 0 && d) d[0] += 1; }

__global__ void k_flag(uint32_t *d, uint32_t *flag, uint32_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        d[0] += 1;
        __atomic_store_n(flag, v, __ATOMIC_RELEASE);   // pinned host memory, system scope via the mapping
    }
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

static void report(const char *name, std::vector<double> &v) {
    std::sort(v.begin(), v.end());
    printf("{\"mode\": \"%s\", \"p50_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", name, v[v.size() / 2], v[v.size() / 10],
           v[v.size() * 9 / 10]);
}

int main() {
    CHK(hipSetDevice(0));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *d;
    CHK(hipMalloc(&d, 64));
    CHK(hipMemset(d, 0, 64));
    uint32_t *hflag, *dflag;
    CHK(hipHostMalloc((void **)&hflag, 64, hipHostMallocMapped));
    CHK(hipHostGetDevicePointer((void **)&dflag, hflag, 0));
    hipEvent_t ev;
    CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int R = 2000;
    for (int i = 0; i < 200; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
    CHK(hipStreamSynchronize(s));
    std::vector<double> t;
    for (int i = 0; i < R; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        hipStreamSynchronize(s);
        t.push_back(us(a, clk::now()));
    }
    report("stream_sync", t);
    t.clear();
    for (int i = 0; i < R; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        hipEventRecord(ev, s);
        hipEventSynchronize(ev);
        t.push_back(us(a, clk::now()));
    }
    report("event_sync", t);
    t.clear();
    volatile uint32_t *vf = hflag;
    for (int i = 0; i < R; i++) {
        const uint32_t v = (uint32_t)i + 1;
        auto a = clk::now();
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, d, dflag, v);
        auto lim = a + std::chrono::milliseconds(200);
        while (*vf != v)
            if (clk::now() > lim) { printf("spin_flag: timeout\n"); return 1; }
        t.push_back(us(a, clk::now()));
    }
    CHK(hipStreamSynchronize(s));
    report("spin_flag", t);
    t.clear();
    for (int i = 0; i < R; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        hipStreamSynchronize(s);
        t.push_back(us(a, clk::now()));
    }
    report("two_kernels", t);
    t.clear();
    for (int i = 0; i < R; i++) {
        const uint32_t v = 0x10000u + (uint32_t)i;
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, d, dflag, v);
        auto lim = a + std::chrono::milliseconds(200);
        while (*vf != v)
            if (clk::now() > lim) { printf("two_kernels_spin: timeout\n"); return 1; }
        t.push_back(us(a, clk::now()));
    }
    CHK(hipStreamSynchronize(s));
    report("two_kernels_spin", t);
    t.clear();
    for (int i = 0; i < R; i++) {
        const uint32_t v = 0x20000u + (uint32_t)i;
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        if (hipStreamWriteValue32(s, dflag, v, 0) != hipSuccess) { printf("write_value unsupported\n"); break; }
        auto lim = a + std::chrono::milliseconds(200);
        while (*vf != v)
            if (clk::now() > lim) { printf("write_value: timeout\n"); return 1; }
        t.push_back(us(a, clk::now()));
    }
    CHK(hipStreamSynchronize(s));
    if (!t.empty()) report("write_value", t);
    return 0;
}

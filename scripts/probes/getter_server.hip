// Round trip of one 8 KB row (V = 1000 merged HighestBefore) from HBM to a
// host thread, three ways (input to the single-row getters):
//   launch_only   host time of the launch call alone
//   row_launch    one launch per row: 256 threads load the row, store it to
//                 pinned memory, system fence, tag; the host spins on the tag
//   row_server    a resident one-workgroup kernel on its own stream polls a
//                 request word in pinned memory and answers the same way; it
//                 leaves on a stop word, after an idle time, or at a deadline
// hipcc --offload-arch=gfx950 -O2 -o getter_server getter_server.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint32_t kRowWords = 2000;   // 8 KB

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(256) k_row(const uint32_t *plane, uint32_t ev, uint32_t *out, uint32_t *tag, uint32_t v) {
    const uint4 *src = reinterpret_cast<const uint4 *>(plane + (uint64_t)ev * kRowWords);
    uint4 r[2];
    const uint32_t n4 = kRowWords / 4;
    for (uint32_t i = 0; i < 2; i++) {
        const uint32_t k = threadIdx.x + i * 256;
        if (k < n4) r[i] = src[k];
    }
    for (uint32_t i = 0; i < 2; i++) {
        const uint32_t k = threadIdx.x + i * 256;
        if (k < n4) reinterpret_cast<uint4 *>(out)[k] = r[i];
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(tag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// req[0] = request number (0: none yet), req[1] = event, req[2] = stop
__global__ void __launch_bounds__(256) k_server(const uint32_t *plane, const uint32_t *req, uint32_t *out, uint32_t *tag,
                                                uint64_t budget_ticks, uint64_t idle_ticks, uint32_t n_ev) {
    __shared__ uint32_t s_req, s_ev, s_go;
    uint32_t seen = 0;
    uint64_t last = wall_clock64();
    const uint64_t deadline = last + budget_ticks;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t q = 0, stop = 0;
            uint64_t now;
            for (;;) {
                q = ld_sys(req);
                stop = ld_sys(req + 2);
                now = wall_clock64();
                if (q != seen || stop || now > deadline || now - last > idle_ticks) break;
                __builtin_amdgcn_s_sleep(1);
            }
            s_go = (q != seen && !stop && now <= deadline) ? 1u : 0u;
            s_req = q;
            s_ev = ld_sys(req + 1);
        }
        __syncthreads();
        if (!s_go) break;   // every thread of the workgroup leaves together
        const uint32_t q = s_req, ev = s_ev < n_ev ? s_ev : 0u;
        seen = q;
        const uint4 *src = reinterpret_cast<const uint4 *>(plane + (uint64_t)ev * kRowWords);
        uint4 r[2];
        const uint32_t n4 = kRowWords / 4;
        for (uint32_t i = 0; i < 2; i++) {
            const uint32_t k = threadIdx.x + i * 256;
            if (k < n4) r[i] = src[k];
        }
        for (uint32_t i = 0; i < 2; i++) {
            const uint32_t k = threadIdx.x + i * 256;
            if (k < n4) reinterpret_cast<uint4 *>(out)[k] = r[i];
        }
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(tag, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = wall_clock64();
        __syncthreads();
    }
}


// one 8-byte poll per iteration: req64 = {request number, event}; number
// 0xFFFFFFFF = stop
__global__ void __launch_bounds__(256) k_server2(const uint32_t *plane, const uint64_t *req, uint32_t *out, uint32_t *tag,
                                                 uint64_t budget_ticks, uint64_t idle_ticks, uint32_t sleep,
                                                 uint32_t n_ev) {
    __shared__ uint32_t s_req, s_ev, s_go;
    uint32_t seen = 0;
    uint64_t last = wall_clock64();
    const uint64_t deadline = last + budget_ticks;
    for (;;) {
        if (threadIdx.x == 0) {
            uint64_t w;
            uint64_t now;
            for (;;) {
                w = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                now = wall_clock64();
                if ((uint32_t)w != seen || now > deadline || now - last > idle_ticks) break;
                if (sleep) __builtin_amdgcn_s_sleep(1);
            }
            const uint32_t q = (uint32_t)w;
            s_go = (q != seen && q != 0xFFFFFFFFu && now <= deadline) ? 1u : 0u;
            s_req = q;
            s_ev = (uint32_t)(w >> 32);
        }
        __syncthreads();
        if (!s_go) break;
        const uint32_t q = s_req, ev = s_ev < n_ev ? s_ev : 0u;
        seen = q;
        const uint4 *src = reinterpret_cast<const uint4 *>(plane + (uint64_t)ev * kRowWords);
        uint4 r[2];
        const uint32_t n4 = kRowWords / 4;
        for (uint32_t i = 0; i < 2; i++) {
            const uint32_t k = threadIdx.x + i * 256;
            if (k < n4) r[i] = src[k];
        }
        for (uint32_t i = 0; i < 2; i++) {
            const uint32_t k = threadIdx.x + i * 256;
            if (k < n4) reinterpret_cast<uint4 *>(out)[k] = r[i];
        }
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(tag, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = wall_clock64();
        __syncthreads();
    }
}

// the empty kernel with the same completion (dispatch + flag landing)
__global__ void k_flag(uint32_t *tag, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(tag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

static void report(const char *name, std::vector<double> &v) {
    std::sort(v.begin(), v.end());
    printf("{\"mode\": \"%s\", \"p50_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"max_us\": %.1f, \"n\": %zu}\n", name,
           v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10], v.back(), v.size());
}

int main() {
    CHK(hipSetDevice(0));
    hipStream_t s, srv;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CHK(hipStreamCreateWithPriority(&srv, hipStreamNonBlocking, hi));
    const uint32_t NE = 5000;
    uint32_t *plane;
    CHK(hipMalloc(&plane, 4ull * kRowWords * NE));
    CHK(hipMemset(plane, 0x5A, 4ull * kRowWords * NE));
    uint32_t *hbuf, *dbuf;   // [0..kRowWords) row, [kRowWords] tag, [kRowWords + 16 ..] requests
    CHK(hipHostMalloc((void **)&hbuf, 4ull * 8192, hipHostMallocMapped));
    CHK(hipHostGetDevicePointer((void **)&dbuf, hbuf, 0));
    memset(hbuf, 0, 4ull * 8192);
    volatile uint32_t *vtag = hbuf + kRowWords;
    volatile uint32_t *vreq = hbuf + kRowWords + 16;
    int rate_khz = 0;
    CHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    printf("{\"wall_clock_khz\": %d, \"priority_range\": [%d, %d]}\n", rate_khz, lo, hi);
    const int R = 3000;
    std::vector<double> t, tl;
    uint32_t v = 0;
    for (int i = 0; i < 300; i++) hipLaunchKernelGGL(k_row, dim3(1), dim3(256), 0, s, plane, 0, dbuf, dbuf + kRowWords, ++v);
    CHK(hipStreamSynchronize(s));
    for (int i = 0; i < R; i++) {
        const uint32_t ev = (uint32_t)(i * 7919u) % NE;
        ++v;
        auto a = clk::now();
        hipLaunchKernelGGL(k_row, dim3(1), dim3(256), 0, s, plane, ev, dbuf, dbuf + kRowWords, v);
        auto b = clk::now();
        auto lim = a + std::chrono::milliseconds(200);
        while (*vtag != v)
            if (clk::now() > lim) { printf("row_launch: timeout\n"); return 1; }
        t.push_back(us(a, clk::now()));
        tl.push_back(us(a, b));
    }
    CHK(hipStreamSynchronize(s));
    report("launch_only", tl);
    report("row_launch", t);
    // the server: a 2 s deadline, 50 ms idle
    const uint64_t tick_per_us = (uint64_t)rate_khz / 1000;
    t.clear();
    vtag[0] = 0;
    vreq[0] = 0;
    vreq[2] = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipLaunchKernelGGL(k_server, dim3(1), dim3(256), 0, srv, plane, dbuf + kRowWords + 16, dbuf, dbuf + kRowWords,
                       3000000ull * tick_per_us, 50000ull * tick_per_us, NE);
    uint32_t q = 0;
    bool ok = true;
    for (int i = 0; i < R && ok; i++) {
        const uint32_t ev = (uint32_t)(i * 7919u) % NE;
        ++q;
        auto a = clk::now();
        vreq[1] = ev;
        std::atomic_thread_fence(std::memory_order_release);
        vreq[0] = q;
        auto lim = a + std::chrono::milliseconds(200);
        while (*vtag != q)
            if (clk::now() > lim) { printf("row_server: timeout at %d\n", i); ok = false; break; }
        if (ok) t.push_back(us(a, clk::now()));
    }
    vreq[2] = 1;   // stop
    std::atomic_thread_fence(std::memory_order_seq_cst);
    CHK(hipStreamSynchronize(srv));
    if (!t.empty()) report("row_server", t);
    // a launch on the ordinary stream while the server runs (queue sharing check)
    t.clear();
    vreq[0] = 0;
    vreq[2] = 0;
    vtag[0] = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipLaunchKernelGGL(k_server, dim3(1), dim3(256), 0, srv, plane, dbuf + kRowWords + 16, dbuf, dbuf + kRowWords,
                       2000000ull * tick_per_us, 20000ull * tick_per_us, NE);
    for (int i = 0; i < 200; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_row, dim3(1), dim3(256), 0, s, plane, 1, dbuf + 4096, dbuf + 4096 + kRowWords, 0x10000u + i);
        CHK(hipStreamSynchronize(s));
        t.push_back(us(a, clk::now()));
    }
    vreq[2] = 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    CHK(hipStreamSynchronize(srv));
    report("other_stream_launch_sync_with_server_resident", t);
    // flag only
    t.clear();
    for (int i = 0; i < R; i++) {
        ++v;
        auto a = clk::now();
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, dbuf + kRowWords, v);
        auto lim = a + std::chrono::milliseconds(200);
        while (*vtag != v)
            if (clk::now() > lim) { printf("flag: timeout\n"); return 1; }
        t.push_back(us(a, clk::now()));
    }
    CHK(hipStreamSynchronize(s));
    report("flag_launch", t);
    // server2: one 8-byte poll, with and without s_sleep
    volatile uint64_t *vreq64 = reinterpret_cast<volatile uint64_t *>(hbuf + kRowWords + 32);
    const uint64_t *dreq64 = reinterpret_cast<const uint64_t *>(dbuf + kRowWords + 32);
    for (uint32_t sl = 0; sl < 2; sl++) {
        t.clear();
        vtag[0] = 0;
        *vreq64 = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        hipLaunchKernelGGL(k_server2, dim3(1), dim3(256), 0, srv, plane, dreq64, dbuf, dbuf + kRowWords,
                           3000000ull * tick_per_us, 50000ull * tick_per_us, sl, NE);
        q = 0;
        ok = true;
        for (int i = 0; i < R && ok; i++) {
            const uint32_t ev = (uint32_t)(i * 7919u) % NE;
            ++q;
            auto a = clk::now();
            *vreq64 = ((uint64_t)ev << 32) | q;
            auto lim = a + std::chrono::milliseconds(200);
            while (*vtag != q)
                if (clk::now() > lim) { printf("row_server2: timeout at %d\n", i); ok = false; break; }
            if (ok) t.push_back(us(a, clk::now()));
        }
        std::vector<double> t2;
        // other-stream work while this server is resident
        for (int i = 0; i < 200 && ok; i++) {
            auto a = clk::now();
            hipLaunchKernelGGL(k_row, dim3(1), dim3(256), 0, s, plane, 1, dbuf + 4096, dbuf + 4096 + kRowWords, 0x20000u + i);
            CHK(hipStreamSynchronize(s));
            t2.push_back(us(a, clk::now()));
        }
        *vreq64 = 0xFFFFFFFFull;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        CHK(hipStreamSynchronize(srv));
        if (!t.empty()) report(sl ? "row_server2_sleep" : "row_server2_busy", t);
        if (!t2.empty()) report(sl ? "other_stream_with_server2_sleep" : "other_stream_with_server2_busy", t2);
    }
    // the same other-stream work without a server
    t.clear();
    for (int i = 0; i < 200; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_row, dim3(1), dim3(256), 0, s, plane, 1, dbuf + 4096, dbuf + 4096 + kRowWords, 0x30000u + i);
        CHK(hipStreamSynchronize(s));
        t.push_back(us(a, clk::now()));
    }
    report("other_stream_no_server", t);
    return 0;
}

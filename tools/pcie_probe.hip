// Microbenchmark (diagnostic, not product code): how device -> host bytes move fastest on this
// box -- hipMemcpyAsync D2H alone, D2H on two streams, D2H concurrent with H2D, and a kernel storing
// 16 B per lane straight into pinned host memory (zero-copy) -- for the record cursor (ppg_cursor).
//   hipcc --offload-arch=gfx950 -O3 tools/pcie_probe.hip -o /tmp/pcie_probe && /tmp/pcie_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <chrono>
#include <string.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void store_host(const uint4 *src, uint4 *dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t N = (size_t)4 << 30;
    uint8_t *d1, *d2, *h1, *h2;
    CK(hipMalloc(&d1, N)); CK(hipMalloc(&d2, N));
    CK(hipHostMalloc(&h1, N, hipHostMallocDefault)); CK(hipHostMalloc(&h2, N, hipHostMallocDefault));
    CK(hipMemset(d1, 1, N)); CK(hipMemset(d2, 2, N));
    memset(h1, 0, N); memset(h2, 0, N);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int rep = 0; rep < 2; rep++) {
        double t = now();
        CK(hipMemcpyAsync(h1, d1, N, hipMemcpyDeviceToHost, s1)); CK(hipStreamSynchronize(s1));
        printf("{\"case\": \"D2H one stream\", \"GBps\": %.1f}\n", N / (now() - t) / 1e9);
        t = now();
        CK(hipMemcpyAsync(h1, d1, N, hipMemcpyDeviceToHost, s1)); CK(hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2));
        printf("{\"case\": \"D2H two streams (total)\", \"GBps\": %.1f}\n", 2 * N / (now() - t) / 1e9);
        t = now();
        CK(hipMemcpyAsync(h1, d1, N, hipMemcpyDeviceToHost, s1)); CK(hipMemcpyAsync(d2, h2, N, hipMemcpyHostToDevice, s2));
        CK(hipStreamSynchronize(s1)); double t1 = now() - t; CK(hipStreamSynchronize(s2)); double t2 = now() - t;
        printf("{\"case\": \"D2H + H2D concurrently\", \"D2H_done_s\": %.3f, \"both_done_s\": %.3f, \"D2H_GBps\": %.1f}\n", t1, t2, N / t1 / 1e9);
        for (int g : {1024, 4096, 16384}) {
            t = now();
            hipLaunchKernelGGL(store_host, dim3(g), dim3(256), 0, s1, (const uint4 *)d1, (uint4 *)h1, N / 16);
            CK(hipStreamSynchronize(s1));
            printf("{\"case\": \"kernel stores to pinned host, %d blocks\", \"GBps\": %.1f}\n", g, N / (now() - t) / 1e9);
        }
        // 4 MiB chunks, 1024 copies on one stream (the cursor's per-chunk pattern)
        t = now();
        for (size_t o = 0; o < N; o += (4 << 20)) CK(hipMemcpyAsync(h1 + o, d1 + o, 4 << 20, hipMemcpyDeviceToHost, s1));
        CK(hipStreamSynchronize(s1));
        printf("{\"case\": \"D2H as 1024 x 4 MiB copies\", \"GBps\": %.1f}\n", N / (now() - t) / 1e9);
    }
    return 0;
}

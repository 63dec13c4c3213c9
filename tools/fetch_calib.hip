// tools/fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE for the access widths the inflate
// kernel uses (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a 16-B-per-lane streaming read; other
// widths are uncalibrated).  Each kernel reads a known number of bytes from a 4 GiB buffer (16x the
// Infinity Cache, so nothing is served on-die from an earlier pass), one dispatch per pattern:
//   k_stream16  16 B per lane, coalesced (the guide's calibrated case)             bytes = 4 GiB
//   k_stream4   4 B per lane, coalesced (global_load_lds_dword: the compressed stream) bytes = 4 GiB
//   k_scatter4  4 B per lane, every lane its own 128-B line (the far loads' worst case)
//               bytes read = lanes x 4, lines touched = lanes x 128
//   k_window4   4 B per lane, 64 lanes gather inside a 32 KiB window that slides 64 B per step
//               (the far loads' actual shape: recent output of the same wave)
// Run: rocprofv3 --pmc FETCH_SIZE -d <dir> -o pmc --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_fill(uint32_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] = (uint32_t)i * 2654435761u;
}

__global__ void k_stream16(const uint4 *p, uint64_t n, uint32_t *sink) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x12345678u) sink[0] = a;
}

__global__ void k_stream4(const uint32_t *p, uint64_t n, uint32_t *sink) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) a ^= p[i];
    if (a == 0x12345678u) sink[0] = a;
}

// lane t of the grid reads the first dword of line t * stride (stride 128 B lines)
__global__ void k_scatter4(const uint32_t *p, uint64_t lines, uint32_t *sink) {
    uint32_t a = 0;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < lines; t += (uint64_t)gridDim.x * 256) a ^= p[t * 32];
    if (a == 0x12345678u) sink[0] = a;
}

// one wave per 4 MiB region: step s reads 64 dwords at pseudo-random offsets in the 32 KiB before
// position 32768 + 64 s (each region read as a sliding window, like a chunk's far references)
__global__ void k_window4(const uint8_t *p, uint64_t region, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t base = (blockIdx.x * 4ull + (threadIdx.x >> 6)) * region;
    uint32_t a = 0, h = lane * 0x9E3779B9u + blockIdx.x;
    for (uint64_t pos = 32768; pos + 64 <= region; pos += 64) {
        h = h * 1664525u + 1013904223u;
        const uint64_t off = pos - 1 - (h >> 17);          // within the last 32 KiB
        a ^= *(const uint32_t *)(p + base + (off & ~3ull));
    }
    if (a == 0x12345678u) sink[0] = a;
}

int main() {
    const uint64_t bytes = 4ull << 30;
    uint8_t *p;
    uint32_t *sink;
    CHK(hipMalloc(&p, bytes));
    CHK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint32_t *)p, bytes / 4);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float ms;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, (const uint4 *)p, bytes / 16, sink);
    hipEventRecord(e1);
    CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_stream16 read %llu bytes in %.3f ms (%.1f GB/s)\n", (unsigned long long)bytes, ms, bytes / ms / 1e6);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_stream4, dim3(8192), dim3(256), 0, 0, (const uint32_t *)p, bytes / 4, sink);
    hipEventRecord(e1);
    CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_stream4 read %llu bytes in %.3f ms (%.1f GB/s)\n", (unsigned long long)bytes, ms, bytes / ms / 1e6);
    const uint64_t lines = bytes / 128;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_scatter4, dim3(8192), dim3(256), 0, 0, (const uint32_t *)p, lines, sink);
    hipEventRecord(e1);
    CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_scatter4 read %llu dwords from %llu distinct 128-B lines (%llu B of lines) in %.3f ms\n",
           (unsigned long long)lines, (unsigned long long)lines, (unsigned long long)(lines * 128), ms);
    const uint64_t region = 4ull << 20;   // 1024 regions of 4 MiB: 256 blocks x 4 waves
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_window4, dim3((unsigned)(bytes / region / 4)), dim3(256), 0, 0, p, region, sink);
    hipEventRecord(e1);
    CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms, e0, e1);
    const uint64_t steps = (region - 32768) / 64, nwaves = bytes / region;
    printf("k_window4 %llu waves x %llu steps x 64 dwords = %llu dword reads over %llu B of regions in %.3f ms\n",
           (unsigned long long)nwaves, (unsigned long long)steps, (unsigned long long)(nwaves * steps * 64),
           (unsigned long long)bytes, ms);
    CHK(hipFree(p));
    return 0;
}

// Microbenchmark (diagnostic, not product code): cycles per token of the inflate kernel's scalar
// walk loop (walk_asm in ppg_inflate.hip: v_readlane, s_lshr m0, s_add, s_and, v_writelane,
// s_cbranch), alone on its SIMD vs with 8 waves per SIMD, and the same chain with two
// independent walks interleaved (what a second speculative walk would overlap).
//   hipcc --offload-arch=gfx950 -O3 tools/walk_lat.hip -o /tmp/walk_lat && /tmp/walk_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

// one walk over a span whose candidate at lane s is a token of (s % 5) + 3 bits and 1 byte
__device__ __forceinline__ void walk1(uint32_t vt, uint32_t &vtin, uint32_t &X) {
    uint32_t t, tmp;
    asm volatile(
        "1:\n\t"
        "v_readlane_b32 %[t], %[vt], %[X]\n\t"
        "s_lshr_b32 m0, %[X], 8\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1C0C0\n\t"
        "v_writelane_b32 %[vtin], %[t], m0\n\t"
        "s_cbranch_scc0 1b"
        : [vtin] "+v"(vtin), [X] "+s"(X), [t] "=&s"(t), [tmp] "=&s"(tmp)
        : [vt] "v"(vt)
        : "m0", "scc");
}

// the walk without placing tokens (v_writelane): what the per-token chain costs without it
__device__ __forceinline__ void walk_nowrite(uint32_t vt, uint32_t &X) {
    uint32_t t, tmp;
    asm volatile(
        "1:\n\t"
        "v_readlane_b32 %[t], %[vt], %[X]\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1C0C0\n\t"
        "s_cbranch_scc0 1b"
        : [X] "+s"(X), [t] "=&s"(t), [tmp] "=&s"(tmp)
        : [vt] "v"(vt)
        : "scc");
}

// the walk recording chosen candidates in a 64-bit mask instead of placing tokens
__device__ __forceinline__ void walk_mask(uint32_t vt, uint64_t &M, uint32_t &X) {
    uint32_t t, tmp;
    asm volatile(
        "1:\n\t"
        "v_readlane_b32 %[t], %[vt], %[X]\n\t"
        "s_bitset1_b64 %[M], %[X]\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1C0C0\n\t"
        "s_cbranch_scc0 1b"
        : [X] "+s"(X), [M] "+s"(M), [t] "=&s"(t), [tmp] "=&s"(tmp)
        : [vt] "v"(vt)
        : "scc");
}

// two independent walks, their instructions interleaved (same loop trip count assumed)
__device__ __forceinline__ void walk2(uint32_t vt, uint32_t &vtin, uint32_t &vtin2, uint32_t &X, uint32_t &Y) {
    uint32_t t, u, tmp, tmq;
    asm volatile(
        "1:\n\t"
        "v_readlane_b32 %[t], %[vt], %[X]\n\t"
        "v_readlane_b32 %[u], %[vt], %[Y]\n\t"
        "s_lshr_b32 m0, %[X], 8\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_add_u32 %[Y], %[u], %[Y]\n\t"
        "v_writelane_b32 %[vtin], %[t], m0\n\t"
        "s_lshr_b32 m0, %[Y], 8\n\t"
        "s_and_b32 %[tmq], %[Y], 0x1C0C0\n\t"
        "s_and_b32 %[tmp], %[X], 0x1C0C0\n\t"
        "v_writelane_b32 %[vtin2], %[u], m0\n\t"
        "s_cbranch_scc0 1b"
        : [vtin] "+v"(vtin), [vtin2] "+v"(vtin2), [X] "+s"(X), [Y] "+s"(Y), [t] "=&s"(t), [u] "=&s"(u),
          [tmp] "=&s"(tmp), [tmq] "=&s"(tmq)
        : [vt] "v"(vt)
        : "m0", "scc");
}

__global__ __launch_bounds__(64) void k(int iters, int mode, unsigned long long *cyc, unsigned long long *tok) {
    const uint32_t lane = threadIdx.x;
    const uint32_t vt = ((lane % 5) + 3) | (1u << 8);   // bits, 1 byte each
    uint32_t vtin = 0, vtin2 = 0, sink = 0;
    unsigned long long n = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        uint32_t X = (uint32_t)(i & 3), Y = (uint32_t)((i + 1) & 3);
        if (mode == 0) {
            walk1(vt, vtin, X);
            n += 1;
        } else if (mode == 2) {
            walk_nowrite(vt, X);
            n += 1;
        } else if (mode == 3) {
            uint64_t M = 0;
            walk_mask(vt, M, X);
            sink += (uint32_t)M;
            n += 1;
        } else {
            walk2(vt, vtin, vtin2, X, Y);
            n += 2;
        }
        sink += X + Y;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        atomicAdd(cyc, (unsigned long long)(t1 - t0));
        atomicAdd(tok, n);
    }
    if (sink == 0x12345678u) cyc[1] = vtin + vtin2;   // keep results alive
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 32);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char *names[] = {"one walk (6 instr/token)", "two interleaved walks (per walk)", "no writelane (4 instr/token)",
                           "mask instead of writelane (5 instr/token)"};
    for (int mode = 0; mode < 4; mode++) {
        for (int waves_per_cu : {1, 4, 32}) {
            hipMemset(d, 0, 32);
            const int iters = 20000;
            hipLaunchKernelGGL(k, dim3(cus * waves_per_cu), dim3(64), 0, 0, iters, mode, d, d + 2);
            hipDeviceSynchronize();
            unsigned long long h[4];
            hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
            // ~ (64 - start) / avg bits ~ 12.8 tokens per walk: tokens per walk measured on the host
            // side as lanes visited; here report cycles per walk per wave
            printf("{\"mode\": \"%s\", \"waves_per_cu\": %d, \"cycles_per_walk\": %.1f}\n", names[mode], waves_per_cu,
                   (double)h[0] / (double)h[2]);
        }
    }
    return 0;
}

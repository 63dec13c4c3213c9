// tools/lanesel_check.hip — checks that gfx950's v_readlane / v_writelane use only bits [5:0] of
// their lane select (the inflate walk relies on it: DESIGN.md §4).  Build and run on the GPU box:
//   hipcc --offload-arch=gfx950 -O2 tools/lanesel_check.hip -o /tmp/lanesel && /tmp/lanesel
// Expected: lane select 0x40 reads lane 0, 0x41 lane 1, 0x1c5 / 0xffffff05 / 0x12345 lane 5.
#include <hip/hip_runtime.h>
#include <stdio.h>
extern "C" __device__ int llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane");
__global__ void k(const unsigned *sel, int *out, int n) {
    int lane = threadIdx.x;
    for (int i = 0; i < n; i++) {
        unsigned s = __builtin_amdgcn_readfirstlane(sel[i]);
        int r = __builtin_amdgcn_readlane(lane * 10 + 7, (int)s);
        int w = llvm_writelane(1000 + i, (int)s, -1);
        unsigned long long b = __ballot(w != -1);
        if (lane == 0) { out[3 * i] = r; out[3 * i + 1] = (int)(b & 0xffffffff); out[3 * i + 2] = (int)(b >> 32); }
    }
}
int main() {
    unsigned hs[8] = {0, 5, 63, 64, 65, 0x1C5, 0xFFFFFF05u, 0x12345u};
    unsigned *ds; int *dout; int ho[24];
    hipMalloc(&ds, sizeof hs); hipMalloc(&dout, sizeof ho);
    hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dout, 8);
    hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
    for (int i = 0; i < 8; i++) printf("sel %#x: readlane -> %d (lane %d)  writelane mask %08x%08x\n", hs[i], ho[3*i], (ho[3*i]-7)/10, ho[3*i+2], ho[3*i+1]);
    return 0;
}

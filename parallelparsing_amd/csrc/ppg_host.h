// ppg_host.h — host-side types shared by the translation units of libppgpu.so
// (ppg_api.cpp: C ABI, index I/O, shards, ingest; ppg_index_gpu.cpp: GPU CreateIndex).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include <algorithm>

#include "../../include/ppgpu.h"
#include "ppg_device.h"

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "ppgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return PPG_DEVICE_ERROR;                                                       \
        }                                                                                  \
    } while (0)

namespace {
constexpr int kWin = PPG_WINSIZE;
// census capacity: one stored newline per this many output bytes (+64) per chunk; FASTQ lines
// average well above it (150 bp Generator records: ~97 B), chunks that overflow fall back to a scan
constexpr int kNlBytesPerEntry = 64;
constexpr int kChunk = PPG_CHUNK;
}

struct PpgPoint {                       // Common/Index.cs:51-82
    int64_t output = 0;                 // offset in the uncompressed stream
    int64_t input = 0;                  // offset of the first full byte in the .gz
    int32_t bits = 0;                   // unused bits (1-7) of byte input-1, or 0
    std::vector<uint8_t> offset;        // bytes since the last '@' (the partial record)
};

struct ppg_index {
    int32_t chunk_max_bytes = 0;
    std::vector<PpgPoint> pts;
    // Point.Window (the preceding 32 KiB of output, oldest first) of point i at i * kWin: one
    // contiguous array, so a range of chunks ships its windows to the GPU in one copy
    std::vector<uint8_t> windows;
    const uint8_t *win(size_t i) const { return windows.data() + i * kWin; }
    // side points (ppg_index_build_gpu_side; not part of the .gzi): block starts inside chunks,
    // absolute bit / output and their 32 KiB windows, for ppg_shard_set_split
    std::vector<int64_t> side_bit, side_out;
    std::vector<uint8_t> side_win;

    // Index.AddPoint (Common/Index.cs:24-48)
    void add_point(int bits, int64_t input, int64_t output, uint32_t left, const uint8_t *circ,
                   const uint8_t *off, size_t off_len) {
        if (pts.empty()) {
            chunk_max_bytes = (int32_t)output;
        } else {
            int32_t sz = (int32_t)((uint32_t)(int32_t)output - (uint32_t)(int32_t)pts.back().output);
            chunk_max_bytes = std::max(chunk_max_bytes, sz);
        }
        PpgPoint p;
        p.output = output;
        p.input = input;
        p.bits = bits;
        // oldest bytes (those after the circular write head) first
        windows.insert(windows.end(), circ + (kWin - left), circ + kWin);
        windows.insert(windows.end(), circ, circ + (kWin - left));
        p.offset.assign(off, off + off_len);
        pts.push_back(std::move(p));
    }
};

struct IngestState;   // host-ingest buffers kept across ppg_file_decompress_all calls

struct ppg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t handoff = nullptr;   // ppg_ctx_wait_stream / ppg_stream_wait_ctx
    IngestState *ingest = nullptr;
    int ring_bits = 10;   // inflate history ring: 2^10..2^15 bytes of LDS per wavefront (1 KiB: 32 waves/CU)
    int lit_bits = 8;     // litlen root table: 2^8 entries (codes <= 8 bits: 99.65% of FASTQ tokens)
    double ix_stats[16] = {0};   // timings / counts of the last GPU CreateIndex (ppg_index_build_gpu_stats)
};

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t count) {
        if (p && n >= count) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; }
        n = count;
        return hipMalloc((void **)&p, std::max<size_t>(count, 1) * sizeof(T));
    }
};

struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t n = 0;
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    hipError_t alloc(size_t count) {
        if (p && n >= count) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; }
        n = count;
        return hipHostMalloc((void **)&p, std::max<size_t>(count, 1), hipHostMallocDefault);
    }
};

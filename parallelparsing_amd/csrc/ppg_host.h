// ppg_host.h — host-side types shared by the translation units of libppgpu.so
// (ppg_api.cpp: C ABI, index I/O, shards, ingest; ppg_index_gpu.cpp: GPU CreateIndex).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include <memory>
#include <new>
#include <utility>
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

// allocator whose value-initialisation is default-initialisation: resize() leaves bytes
// uninitialised, so a window array can grow and be filled by one device-to-host copy
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) {}
    template <class U>
    void construct(U *p) noexcept { ::new ((void *)p) U; }
    template <class U, class... A>
    void construct(U *p, A &&...a) { ::new ((void *)p) U(std::forward<A>(a)...); }
};
using ByteVec = std::vector<uint8_t, NoInitAlloc<uint8_t>>;

struct ppg_index {
    int32_t chunk_max_bytes = 0;
    std::vector<PpgPoint> pts;
    // Point.Window (the preceding 32 KiB of output, oldest first) of point i at i * kWin: one
    // contiguous array, so a range of chunks ships its windows to the GPU in one copy
    ByteVec windows;
    const uint8_t *win(size_t i) const { return windows.data() + i * kWin; }
    // side points (ppg_index_build_gpu_side; not part of the .gzi): block starts inside chunks,
    // absolute bit / output and their 32 KiB windows, for ppg_shard_set_split
    std::vector<int64_t> side_bit, side_out;
    ByteVec side_win;

    // Index.AddPoint (Common/Index.cs:24-48)
    void add_point(int bits, int64_t input, int64_t output, uint32_t left, const uint8_t *circ,
                   const uint8_t *off, size_t off_len) {
        // oldest bytes (those after the circular write head) first
        windows.insert(windows.end(), circ + (kWin - left), circ + kWin);
        windows.insert(windows.end(), circ, circ + (kWin - left));
        add_point_fields(bits, input, output, off, off_len);
    }
    // the same without the window (the caller has appended it to `windows` already)
    void add_point_fields(int bits, int64_t input, int64_t output, const uint8_t *off, size_t off_len) {
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
        p.offset.assign(off, off + off_len);
        pts.push_back(std::move(p));
    }
};

struct IngestState;   // host-ingest buffers kept across ppg_file_decompress_all calls
struct ChunkService;  // ppg_decompress_chunk's launch slots and request queue (ppg_chunk.cpp)
ChunkService *chunk_service_new();
void chunk_service_free(ChunkService *svc);

constexpr int kIxStats = 18;   // ppg_index_build_gpu_stats values (parallelparsing_amd.Core.GPU_INDEX_STATS)

struct ppg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t handoff = nullptr;   // ppg_ctx_wait_stream / ppg_stream_wait_ctx
    IngestState *ingest = nullptr;
    ChunkService *chunks = nullptr;
    int ring_bits = 11;   // inflate history ring: 2^10..2^15 bytes of LDS per wavefront (2 KiB: 32 waves/CU)
    int lit_bits = 8;     // litlen root table: 2^8 entries (codes <= 8 bits: 99.65% of FASTQ tokens)
    double ix_stats[kIxStats] = {0};   // timings / counts of the last GPU CreateIndex (ppg_index_build_gpu_stats)
    uint8_t *stage = nullptr;           // pinned device -> host staging (CreateIndex windows), kept across calls
    size_t stage_n = 0;
};

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
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

// DecompressAll state over chunks [first, first+n) of an index (ppg_api.cpp); the cursor and the
// multi-GPU entry points (ppg_multi.cpp) drive it through the functions below.
struct ppg_shard {
    ppg_ctx *ctx = nullptr;
    int32_t first = 0, n = 0;
    // compressed file range [Index[first].Input-1, Index[first+n].Input-1]
    DevBuf<uint8_t> comp_own;
    const uint8_t *comp = nullptr;
    int64_t comp_len = 0;
    uint64_t nwords = 0;
    DevBuf<PpgInflateJob> jobs;
    DevBuf<uint8_t> dicts;
    DevBuf<uint8_t> offs;
    DevBuf<PpgOffsetRef> oref;
    DevBuf<PpgInflateResult> res;
    DevBuf<PpgParseInfo> info;
    DevBuf<uint64_t> base;     // record base within the batch
    DevBuf<uint64_t> total;
    DevBuf<uint8_t> out;
    DevBuf<uint32_t> recs;     // descriptors of every record of the run, shard-global (all batches)
    DevBuf<uint32_t> nls;      // newline census of the inflate flush (PpgInflateJob::nl_off/nl_cap)
    int64_t out_cap = 0;
    std::vector<std::pair<int32_t, int32_t>> batches;   // chunk ranges [b0, b1) relative to first
    std::vector<PpgInflateJob> h_jobs;
    // results of the last run
    std::vector<PpgInflateResult> h_res;
    std::vector<PpgParseInfo> h_info;
    std::vector<int64_t> h_base;   // shard-global record base per chunk
    int64_t total_records = 0;
    float t_inflate = 0, t_parse = 0, t_total = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipStream_t stream = nullptr;   // null: the ctx stream (ppg_file_decompress_all gives each piece shard its own)
    uint64_t *h_tot = nullptr;      // pinned: a batch's record total, read back without a stream sync
    int ran = 0;
    int last_rc = PPG_OK;           // status of the last ppg_shard_run (the count gather forwards it)
    // ppg_shard_set_keys: every batch also writes its records' spot keys here (global record number)
    int64_t *keys_dev = nullptr;
    int64_t keys_cap = 0;
    int keys_written = 0;   // the last successful run filled keys_dev (set by shard_run)
    // split chunks (ppg_shard_set_split): the inflate launch runs sub-jobs, ppg_split_merge folds
    // them back into per-chunk results and census regions
    int32_t nsub = 0;                            // side points in use (0: one wave per chunk)
    int64_t base_byte = 0;                       // file byte of comp[0]
    std::vector<int64_t> h_pout;                 // Output of points first .. first + n
    std::vector<PpgInflateJob> h_sjobs;
    DevBuf<PpgInflateJob> sjobs;
    DevBuf<PpgInflateResult> sres;
    DevBuf<uint32_t> sidx;                      // chunk k = sub-jobs [sidx[k], sidx[k+1])
    std::vector<uint32_t> h_sidx;
    bool lpt = false;                           // the launch runs ljobs: sub-jobs longest first per batch,
    DevBuf<PpgInflateJob> ljobs;                // results in that order, sub-job j's at linv[j]
    DevBuf<uint32_t> linv;
    // one-batch launches whose pieces are materialised from pass-1 symbols (ppg_chunk.cpp): ljobs
    // [0, mat_first) are decoded, [mat_first, nsub + n) materialised with mat_info (launch order)
    uint32_t mat_n = 0, mat_first = 0;
    const uint16_t *mat_sym = nullptr;
    const uint8_t *mat_win = nullptr;
    const PpgMatInfo *mat_info = nullptr;
};

// one chunk of a shard: its Points, its window and where file byte from.Input-1 sits in comp
struct ChunkSpec {
    const PpgPoint *from, *to;
    const uint8_t *window;
    int64_t comp_byte;
    bool last;                          // `to` is the index's final Point (R-E5 end not checkable)
};
int shard_prepare_specs(ppg_shard *sh, const ChunkSpec *spec, int32_t n, const uint8_t *comp, int64_t comp_len,
                        int64_t out_capacity, hipStream_t s, const uint8_t *windows_contig);
int shard_prepare(ppg_shard *sh, const ppg_index *ix, int32_t first, int32_t n, const uint8_t *comp, int64_t comp_len,
                  int64_t out_capacity, hipStream_t s);
hipStream_t shard_stream(const ppg_shard *sh);
void shard_reset(ppg_shard *sh);
int batch_launch(ppg_shard *sh, int32_t b0, int32_t b1);
int batch_collect(ppg_shard *sh, int32_t b0, int32_t b1, float &total_ms);
int shard_finish(ppg_shard *sh, float total_ms);
int shard_split_from_index(ppg_shard *sh, const ppg_index *ix, int32_t first, int32_t n);
int shard_set_split_impl(ppg_shard *sh, int32_t nsub, const int64_t *bit, const int64_t *output,
                         const uint8_t *windows, bool lpt);
int shard_reserve(ppg_shard *sh, const ppg_index *ix, int32_t first,
                  const std::vector<std::pair<int32_t, int32_t>> &ranges, bool split);
bool pread_parallel(int fd, uint8_t *dst, int64_t off, int64_t len, int threads);

// collectives of a ppg_comm beyond the count gather (ppg_comm.cpp), used by ppg_pairs.hip
int comm_size(const ppg_comm *c, int32_t *rank, int32_t *nranks);
int comm_device(const ppg_comm *c);   // -1: host transport
int comm_all_gather_i64(ppg_comm *c, const int64_t *send, int64_t *recv, size_t n, bool &sent_ok);
int comm_alltoallv_i64(ppg_comm *c, hipStream_t s, const int64_t *send, int64_t *recv, const int64_t *m,
                       bool on_device);
// the RCCL point-to-point entry points of one grouped exchange (ppg_comm.cpp; host_check passes fakes)
struct CommP2P {
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*group_start)();
    ncclResult_t (*group_end)();
    const char *(*err)(ncclResult_t);
};
int comm_grouped_p2p(const CommP2P &f, void *comm, hipStream_t stream, const int64_t *send, int64_t *recv,
                     const int64_t *m, int32_t R, int32_t me, const int64_t *sd, const int64_t *rd);

// ppg_api.cpp — host side of libppgpu.so: the C ABI declared in include/ppgpu.h.
//
//   Index model + CreateIndex      Common/Index.cs, Decompressor/Core.cs:14-131 (serial zlib pass)
//   .gzi Serialize / Deserialize   Common/IndexIO.cs:7-53
//   ppg_ctx                        one GPU, one HIP stream
//   ppg_shard                      DecompressAll over chunks [first, first+n): device-resident
//                                  compressed range + windows + offsets, batched inflate + parse
//   ppg_file_decompress_all        host ingest (LazyFileReader.cs:10-98): pread into pinned
//                                  buffers, H2D on a copy stream overlapped with decoding
//
// No CPU fallback exists for the decode: without a usable gfx950 device every decode entry point
// returns PPG_NO_DEVICE / PPG_DEVICE_ERROR.
#include <hip/hip_runtime.h>
#include <zlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <vector>
#include <string>
#include <algorithm>
#include <memory>
#include <thread>
#include <mutex>
#include <condition_variable>
#include <chrono>
#include <fcntl.h>
#include <unistd.h>

#include "../../include/ppgpu.h"
#include "ppg_device.h"
#include "ppg_host.h"

// launchers (ppg_inflate.hip, ppg_parse.hip)
size_t ppg_inflate_lds_bytes(int ring_bits, int lit_bits);
hipError_t ppg_launch_inflate(hipStream_t s, int ring_bits, int lit_bits, const uint32_t *comp, uint64_t nwords,
                              const PpgInflateJob *jobs, const uint8_t *dicts, uint8_t *out, PpgInflateResult *res,
                              int njobs, uint32_t *nls);
hipError_t ppg_launch_total_to_host(hipStream_t s, const uint64_t *total, uint64_t *host);
hipError_t ppg_launch_parse_count(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  PpgParseInfo *info, uint64_t *base, uint64_t *total, int n, const uint32_t *nls);
hipError_t ppg_launch_materialize(hipStream_t s, const uint16_t *sym, const uint8_t *wins, const PpgMatInfo *mi,
                                  const PpgInflateJob *jobs, uint8_t *out, PpgInflateResult *res, int njobs,
                                  uint32_t *nls);
hipError_t ppg_launch_split_merge(hipStream_t s, const PpgInflateJob *sjobs, const PpgInflateResult *sres,
                                  const uint32_t *inv, const uint32_t *sidx, const uint32_t *snls,
                                  const PpgInflateJob *jobs, PpgInflateResult *res, uint32_t *nls, int n);
hipError_t ppg_launch_parse_emit(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                 const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                 PpgParseInfo *info, const uint64_t *base, const uint32_t *nls, uint32_t *recs,
                                 uint64_t cap, int n);
hipError_t ppg_launch_record_keys(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  const PpgParseInfo *info, const uint64_t *base, const uint32_t *recs, int64_t *keys,
                                  int n);

namespace {

// Byte source read in FileStream.Read(input, 0, CHUNK) steps (Core.cs:41).
struct Source {
    const uint8_t *mem = nullptr;
    int64_t len = 0, pos = 0;
    FILE *f = nullptr;
    int64_t flen = 0;
    size_t read(uint8_t *dst, size_t n) {
        if (f) {
            size_t got = fread(dst, 1, n, f);
            pos += (int64_t)got;
            return got;
        }
        size_t k = (size_t)std::min<int64_t>((int64_t)n, len - pos);
        memcpy(dst, mem + pos, k);
        pos += (int64_t)k;
        return k;
    }
    bool at_end() const { return pos == (f ? flen : len); }
};

// Core.BuildDeflateIndex restated over zlib 1.2.11's inflate(Z_BLOCK).
class IndexBuilder {
  public:
    explicit IndexBuilder(uint32_t chunksize)
        // int recordCounter > uint (chunksize - 8): compared as long (Core.cs:105)
        : threshold_((int64_t)(uint32_t)(chunksize - 8u)) {}

    int build(Source &src, ppg_index &ix) {
        z_stream zs;
        memset(&zs, 0, sizeof zs);
        int ret = inflateInit2(&zs, 47);   // gzip/zlib auto-detect, 32 KiB window (Core.cs:30)
        if (ret != Z_OK) return ret;
        std::unique_ptr<z_stream, int (*)(z_stream *)> guard(&zs, inflateEnd);
        std::vector<uint8_t> in(kChunk), circ(kWin, 0);
        int64_t totin = 0, totout = 0;
        bool have_window = false;   // strm.NextOut != null
        zs.avail_out = 0;
        do {
            zs.avail_in = (uInt)src.read(in.data(), kChunk);
            if (zs.avail_in == 0) return Z_DATA_ERROR;
            zs.next_in = in.data();
            do {
                if (zs.avail_out == 0) {
                    zs.avail_out = kWin;
                    zs.next_out = circ.data();
                    have_window = true;
                }
                const uint32_t out_before = zs.avail_out;
                totin += zs.avail_in;
                totout += zs.avail_out;
                ret = inflate(&zs, Z_BLOCK);
                totin -= zs.avail_in;
                totout -= zs.avail_out;
                switch (ret) {
                    case Z_NEED_DICT: case Z_MEM_ERROR: case Z_DATA_ERROR:
                    case Z_STREAM_ERROR: case Z_BUF_ERROR: case Z_VERSION_ERROR:
                        return ret;                                    // Core.cs:68-74
                    default: break;
                }
                if (have_window) {
                    int rc = scan(circ.data() + (kWin - out_before), out_before - zs.avail_out);
                    if (rc) return rc;
                    const int dt = zs.data_type;
                    if ((dt & 128) && !(dt & 64)) {                   // end of a non-final block
                        if (totout == 0) {
                            ix.add_point(dt & 7, totin, 0, zs.avail_out, circ.data(), nullptr, 0);
                        } else if (records_ > threshold_) {
                            ix.add_point(dt & 7, totin, totout, zs.avail_out, circ.data(), partial_.data(),
                                         partial_.size());
                            records_ = 0;
                        }
                    }
                }
                if (ret == Z_STREAM_END) {
                    if (zs.avail_in != 0 || !src.at_end()) {          // another member (Core.cs:116-122)
                        ret = inflateReset(&zs);
                        if (ret != Z_OK) return ret;
                        continue;
                    }
                    ix.add_point(zs.data_type & 7, totin, totout, zs.avail_out, circ.data(), nullptr, 0);
                    break;
                }
            } while (zs.avail_in != 0);
        } while (ret != Z_STREAM_END);
        return PPG_OK;
    }

  private:
    // the '@' census of Core.cs:79-96: each '@' starts a record and restarts the partial buffer
    int scan(const uint8_t *p, size_t n) {
        for (size_t i = 0; i < n; i++) {
            if (p[i] == '@') {
                records_++;
                partial_.clear();
            }
            if (partial_.size() >= (size_t)kWin) return PPG_INDEX_OUT_OF_RANGE;
            partial_.push_back(p[i]);
        }
        return 0;
    }

    int64_t threshold_;
    int64_t records_ = 0;
    std::vector<uint8_t> partial_;
};

bool write_all(FILE *f, const void *p, size_t n) { return n == 0 || fwrite(p, 1, n, f) == n; }
bool read_all(FILE *f, void *p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

}  // namespace

extern "C" {

int ppg_index_build_mem(const uint8_t *gz, int64_t gz_len, uint32_t chunksize, ppg_index **out) {
    if (!gz || gz_len < 0 || !out) return PPG_ARG_ERROR;
    Source src;
    src.mem = gz;
    src.len = gz_len;
    auto ix = std::make_unique<ppg_index>();
    IndexBuilder b(chunksize);
    int rc = b.build(src, *ix);
    if (rc != PPG_OK) return rc;
    *out = ix.release();
    return PPG_OK;
}

int ppg_index_build_file(const char *gz_path, uint32_t chunksize, ppg_index **out) {
    if (!gz_path || !out) return PPG_ARG_ERROR;
    FILE *f = fopen(gz_path, "rb");
    if (!f) return PPG_IO_ERROR;
    Source src;
    src.f = f;
    fseeko(f, 0, SEEK_END);
    src.flen = ftello(f);
    fseeko(f, 0, SEEK_SET);
    auto ix = std::make_unique<ppg_index>();
    IndexBuilder b(chunksize);
    int rc = b.build(src, *ix);
    fclose(f);
    if (rc != PPG_OK) return rc;
    *out = ix.release();
    return PPG_OK;
}

// IndexIO.Serialize (IndexIO.cs:7-27): i32 0, i32 ChunkMaxBytes, i32 Count, then per point
// i64 Output, i64 Input, i32 Bits, i32 WinLen, u8[WinLen], i32 OffLen, u8[OffLen] (little endian)
int ppg_index_serialize(const ppg_index *ix, const char *path) {
    if (!ix || !path) return PPG_ARG_ERROR;
    FILE *f = fopen(path, "wb");
    if (!f) return PPG_IO_ERROR;
    bool ok = true;
    const int32_t hdr[3] = {0, ix->chunk_max_bytes, (int32_t)ix->pts.size()};
    ok &= write_all(f, hdr, sizeof hdr);
    for (size_t i = 0; i < ix->pts.size(); i++) {
        const auto &p = ix->pts[i];
        const int32_t wl = kWin, ol = (int32_t)p.offset.size();
        ok &= write_all(f, &p.output, 8) && write_all(f, &p.input, 8) && write_all(f, &p.bits, 4);
        ok &= write_all(f, &wl, 4) && write_all(f, ix->win(i), kWin);
        ok &= write_all(f, &ol, 4) && write_all(f, p.offset.data(), p.offset.size());
    }
    ok &= fclose(f) == 0;
    return ok ? PPG_OK : PPG_IO_ERROR;
}

// IndexIO.Deserialize (IndexIO.cs:29-53); ChunkMaxBytes is read back (the C# drops it).
int ppg_index_deserialize(const char *path, ppg_index **out) {
    if (!path || !out) return PPG_ARG_ERROR;
    FILE *f = fopen(path, "rb");
    if (!f) return PPG_IO_ERROR;
    auto ix = std::make_unique<ppg_index>();
    int32_t hdr[3];
    bool ok = read_all(f, hdr, sizeof hdr) && hdr[2] >= 0;
    std::vector<uint8_t> wbuf;
    for (int32_t i = 0; ok && i < hdr[2]; i++) {
        PpgPoint p;
        int32_t wl = 0, ol = 0;
        ok = read_all(f, &p.output, 8) && read_all(f, &p.input, 8) && read_all(f, &p.bits, 4) && read_all(f, &wl, 4) &&
             wl >= 0;
        if (!ok) break;
        wbuf.assign((size_t)std::max(wl, kWin), 0);
        ok = read_all(f, wbuf.data(), (size_t)wl) && read_all(f, &ol, 4) && ol >= 0;
        if (!ok) break;
        p.offset.resize((size_t)ol);
        ok = read_all(f, p.offset.data(), (size_t)ol);
        // inflateSetDictionary(Window, 32768) (Core.cs:158) uses the first 32 KiB
        ix->windows.insert(ix->windows.end(), wbuf.begin(), wbuf.begin() + kWin);
        ix->pts.push_back(std::move(p));
    }
    fclose(f);
    if (!ok) return PPG_IO_ERROR;
    ix->chunk_max_bytes = hdr[1];
    *out = ix.release();
    return PPG_OK;
}

int ppg_index_from_points(int32_t count, const int64_t *output, const int64_t *input, const int32_t *bits,
                          const uint8_t *windows, const int32_t *offset_len, const uint8_t *offsets,
                          int32_t chunk_max_bytes, ppg_index **out) {
    if (count < 0 || !output || !input || !bits || !windows || !offset_len || !out) return PPG_ARG_ERROR;
    auto ix = std::make_unique<ppg_index>();
    ix->chunk_max_bytes = chunk_max_bytes;
    ix->pts.resize((size_t)count);
    ix->windows.assign(windows, windows + (size_t)count * kWin);
    size_t o = 0;
    for (int32_t i = 0; i < count; i++) {
        PpgPoint &p = ix->pts[(size_t)i];
        p.output = output[i];
        p.input = input[i];
        p.bits = bits[i];
        if (offset_len[i] < 0) return PPG_ARG_ERROR;
        p.offset.assign(offsets + o, offsets + o + offset_len[i]);
        o += (size_t)offset_len[i];
    }
    *out = ix.release();
    return PPG_OK;
}

int32_t ppg_index_count(const ppg_index *ix) { return ix ? (int32_t)ix->pts.size() : 0; }
int32_t ppg_index_chunk_max_bytes(const ppg_index *ix) { return ix ? ix->chunk_max_bytes : 0; }

int ppg_index_point(const ppg_index *ix, int32_t i, int64_t *output, int64_t *input, int32_t *bits,
                    int32_t *offset_len) {
    if (!ix || i < 0 || (size_t)i >= ix->pts.size()) return PPG_ARG_ERROR;
    const PpgPoint &p = ix->pts[(size_t)i];
    if (output) *output = p.output;
    if (input) *input = p.input;
    if (bits) *bits = p.bits;
    if (offset_len) *offset_len = (int32_t)p.offset.size();
    return PPG_OK;
}

const uint8_t *ppg_index_window(const ppg_index *ix, int32_t i) {
    if (!ix || i < 0 || (size_t)i >= ix->pts.size()) return nullptr;
    return ix->win((size_t)i);
}

const uint8_t *ppg_index_offset(const ppg_index *ix, int32_t i) {
    if (!ix || i < 0 || (size_t)i >= ix->pts.size()) return nullptr;
    return ix->pts[(size_t)i].offset.data();
}

void ppg_index_free(ppg_index *ix) { delete ix; }

// What the decode kernels can take (ppg_shard_create checks it): Points ordered by Input; per
// chunk an output length below 2^31 together with its offset carry (the kernel and the descriptors
// index a chunk's raw bytes with 32 bits; the reference's (int)(to.Output - from.Output), Core.cs:140,
// breaks at the same size) and a compressed span of fewer than 2^32 - 2^12 bits (the kernel's bit
// reader is 32-bit relative to the 4096-bit line holding the chunk's first bit).
int ppg_index_validate(const ppg_index *ix, int32_t first, int32_t n) {
    if (!ix || first < 0 || n < 0 || (size_t)first + (size_t)n + 1 > ix->pts.size()) return PPG_ARG_ERROR;
    for (int32_t i = 0; i < n; i++) {
        const PpgPoint &from = ix->pts[(size_t)first + i], &to = ix->pts[(size_t)first + i + 1];
        if (from.input < 1 || to.input < from.input || from.bits < 0 || from.bits > 7 || to.bits < 0 || to.bits > 7)
            return PPG_ARG_ERROR;
        const int64_t ulen = to.output - from.output;
        if (ulen > 0 && (uint64_t)ulen + from.offset.size() >= (1ull << 31)) return PPG_UNSUPPORTED;
        const uint64_t b0 = (uint64_t)(8 * from.input - from.bits), b1 = (uint64_t)(8 * to.input);
        if (b1 - (b0 & ~4095ull) >= 0xFFFFF000ull) return PPG_UNSUPPORTED;
    }
    return PPG_OK;
}

const char *ppg_version(void) { return "ppgpu 0.3 gfx950 (wave-per-chunk inflate, 2 KiB LDS history ring, fused newline census)"; }

}  // extern "C"

// ====================================== device ======================================

namespace {

bool device_is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

}  // namespace

extern "C" {

int ppg_device_count(int *n) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    if (n) *n = c;
    return c > 0 ? PPG_OK : PPG_NO_DEVICE;
}

int ppg_open(int device, ppg_ctx **out) {
    if (!out) return PPG_ARG_ERROR;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c == 0) return PPG_NO_DEVICE;
    if (device < 0 || device >= c) return PPG_ARG_ERROR;
    if (!device_is_gfx950(device)) {
        fprintf(stderr, "ppgpu: device %d is not gfx950 (MI355X); this library only carries gfx950 code\n", device);
        return PPG_NO_DEVICE;
    }
    HIPCHK(hipSetDevice(device));
    auto ctx = std::make_unique<ppg_ctx>();
    ctx->device = device;
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    ctx->chunks = chunk_service_new();
    if (const char *rb = getenv("PPG_RING_BITS")) ctx->ring_bits = std::min(15, std::max(10, atoi(rb)));
    if (const char *lb = getenv("PPG_LIT_BITS")) ctx->lit_bits = std::min(9, std::max(8, atoi(lb)));
    if (ppg_inflate_lds_bytes(ctx->ring_bits, ctx->lit_bits) == 0) { ctx->ring_bits = 11; ctx->lit_bits = 8; }
    *out = ctx.release();
    return PPG_OK;
}

}  // extern "C"
static void ingest_free(IngestState *st);
extern "C" {

void ppg_close(ppg_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    ingest_free(ctx->ingest);
    chunk_service_free(ctx->chunks);
    if (ctx->stage) (void)hipHostFree(ctx->stage);
    if (ctx->handoff) (void)hipEventDestroy(ctx->handoff);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void *ppg_ctx_stream(ppg_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// Stream-ordered handoff with a caller's stream (torch's current stream, a C# host's own): one
// event recorded on the producer stream, waited on by the consumer stream -- no host drain.
static int stream_order(ppg_ctx *ctx, hipStream_t producer, hipStream_t consumer) {
    HIPCHK(hipSetDevice(ctx->device));
    if (!ctx->handoff) HIPCHK(hipEventCreateWithFlags(&ctx->handoff, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->handoff, producer));
    HIPCHK(hipStreamWaitEvent(consumer, ctx->handoff, 0));
    return PPG_OK;
}

int ppg_ctx_wait_stream(ppg_ctx *ctx, void *stream) {
    if (!ctx) return PPG_ARG_ERROR;
    return stream_order(ctx, (hipStream_t)stream, ctx->stream);
}

int ppg_stream_wait_ctx(ppg_ctx *ctx, void *stream) {
    if (!ctx) return PPG_ARG_ERROR;
    return stream_order(ctx, ctx->stream, (hipStream_t)stream);
}

}  // extern "C"

// ====================================== shard ======================================
// struct ppg_shard: ppg_host.h

extern "C" {

void ppg_shard_free(ppg_shard *sh) {
    if (!sh) return;
    (void)hipSetDevice(sh->ctx->device);
    for (auto &e : sh->ev) if (e) (void)hipEventDestroy(e);
    if (sh->h_tot) (void)hipHostFree(sh->h_tot);
    delete sh;
}

}  // extern "C"

// (Re)build a shard's per-chunk state for chunks [first, first+n) whose compressed range
// [Index[first].Input-1, Index[first+n].Input-1] is at device pointer comp (4-byte aligned,
// readable 64 bytes past comp_len).  Device buffers are reused when large enough, so a shard can
// be re-prepared piece after piece (ppg_file_decompress_all).
int shard_prepare(ppg_shard *sh, const ppg_index *ix, int32_t first, int32_t n, const uint8_t *comp,
                         int64_t comp_len, int64_t out_capacity, hipStream_t s) {
    const auto &P = ix->pts;
    const int64_t base_byte = P[(size_t)first].input - 1;
    if (base_byte < 0) return PPG_ARG_ERROR;
    if (const int v = ppg_index_validate(ix, first, n); v != PPG_OK) return v;
    if (comp_len != P[(size_t)first + n].input - P[(size_t)first].input + 1) return PPG_ARG_ERROR;
    if (ix->windows.size() < ((size_t)first + n) * kWin) return PPG_ARG_ERROR;
    std::vector<ChunkSpec> spec((size_t)n);
    for (int32_t i = 0; i < n; i++)
        spec[(size_t)i] = ChunkSpec{&P[(size_t)first + i], &P[(size_t)first + i + 1], ix->win((size_t)first + i),
                                    P[(size_t)first + i].input - 1 - base_byte, (size_t)first + i + 2 == P.size()};
    const int rc = shard_prepare_specs(sh, spec.data(), n, comp, comp_len, out_capacity, s,
                                       n ? ix->win((size_t)first) : nullptr);
    if (rc != PPG_OK) return rc;
    // the chunks are one contiguous range of the file: absolute coordinates (ppg_shard_set_split
    // takes side points in file bits and stream output offsets)
    sh->first = first;
    sh->base_byte = base_byte;
    for (int32_t i = 0; i <= n; i++) sh->h_pout[(size_t)i] = P[(size_t)first + i].output;
    return PPG_OK;
}

// The same for any list of chunks, each with its own place in comp (ppg_decompress_chunk gathers
// the slices of unrelated chunks, possibly of different indexes, into one launch).  Coordinates are
// virtual: base_byte 0, h_pout[k] = the chunk's output offset in the (single-batch, when
// out_capacity = 0) output buffer; windows_contig, when non-null, holds the n windows back to back.
int shard_prepare_specs(ppg_shard *sh, const ChunkSpec *spec, int32_t n, const uint8_t *comp, int64_t comp_len,
                        int64_t out_capacity, hipStream_t s, const uint8_t *windows_contig) {
    if (((uintptr_t)comp & 3) != 0) return PPG_ARG_ERROR;
    sh->first = 0;
    sh->n = n;
    sh->base_byte = 0;
    sh->h_pout.resize((size_t)n + 1);
    sh->nsub = 0;
    sh->comp = comp;
    sh->comp_len = comp_len;
    sh->nwords = (uint64_t)(comp_len + 3) / 4;
    sh->ran = 0;
    sh->batches.clear();
    // batches: consecutive chunks whose outputs fit out_capacity (0 = everything at once)
    int64_t total_out = 0;
    for (int32_t i = 0; i < n; i++) total_out += std::max<int64_t>(spec[i].to->output - spec[i].from->output, 0);
    int64_t cap = out_capacity > 0 ? out_capacity : total_out;
    sh->h_jobs.resize((size_t)n);
    int64_t need_max = 0;
    uint64_t nl_batch = 0, nl_need = 0;
    // census capacity: one stored newline per kNlBytesPerEntry output bytes; PPG_NL_BYTES overrides
    // (tests force the overflow fallback with a huge value)
    uint64_t nl_bytes = kNlBytesPerEntry;
    if (const char *e = getenv("PPG_NL_BYTES")) nl_bytes = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    {
        int32_t b0 = 0;
        int64_t pos = 0, bbase = 0;   // output offset of chunk i in the whole list / of its batch
        for (int32_t i = 0; i < n; i++) {
            const PpgPoint &from = *spec[i].from, &to = *spec[i].to;
            int64_t ulen = to.output - from.output;
            if (ulen < 0) ulen = 0;   // Core.cs:145: len < 0 -> nothing produced
            if (pos + ulen - bbase > cap && i > b0) {
                sh->batches.push_back({b0, i});
                need_max = std::max(need_max, pos - bbase);
                b0 = i;
                bbase = pos;
            }
            sh->h_pout[(size_t)i] = pos;
            PpgInflateJob &J = sh->h_jobs[(size_t)i];
            const int64_t cb = spec[i].comp_byte;   // comp offset of file byte from.Input - 1
            J.bit_start = (uint64_t)(8 * (cb + 1) - from.bits);
            J.bit_limit = (uint64_t)(8 * (cb + 1 + to.input - from.input));
            J.out_off = (uint64_t)(pos - bbase);
            J.out_len = (uint64_t)ulen;
            J.dict_off = (uint64_t)i * kWin;
            J.expect_end = spec[i].last ? ~0ull : (uint64_t)(8 * (cb + 1 + to.input - from.input) - to.bits);
            // newline census (offsets relative to the batch, like out_off)
            if (i == b0) nl_batch = 0;
            const uint64_t ncap = nl_bytes >= (1ull << 40) ? 0 : (uint64_t)ulen / nl_bytes + 64;
            J.nl_off = nl_batch;
            J.nl_cap = (uint32_t)std::min<uint64_t>(ncap, 0xFFFFFFFFu);
            nl_batch += J.nl_cap;
            nl_need = std::max(nl_need, nl_batch);
            J.raw_shift = (uint32_t)from.offset.size();
            J.prev_byte = from.offset.empty() ? (uint32_t)'\n' : (uint32_t)from.offset.back();
            J.pad = 0;
            pos += ulen;
        }
        sh->h_pout[(size_t)n] = pos;
        if (n > 0) {
            sh->batches.push_back({b0, n});
            need_max = std::max(need_max, pos - bbase);
        }
    }
    const int64_t out_cap = std::max<int64_t>(need_max, 0);
    HIPCHK(sh->jobs.alloc((size_t)n));
    HIPCHK(hipMemcpyAsync(sh->jobs.p, sh->h_jobs.data(), sizeof(PpgInflateJob) * (size_t)n, hipMemcpyHostToDevice, s));
    // windows and offsets of the chunks' `from` points
    std::vector<PpgOffsetRef> horef((size_t)n);
    std::vector<uint8_t> hoff;
    for (int32_t i = 0; i < n; i++) {
        const PpgPoint &from = *spec[i].from;
        horef[(size_t)i].start = hoff.size();
        horef[(size_t)i].len = (uint32_t)from.offset.size();
        // the offset's own newlines, and whether it alone breaks R-P3 (raw[0] == '\n', "\n\n", NUL)
        uint32_t nl = 0;
        bool bad = false, nul = false;
        for (size_t j = 0; j < from.offset.size(); j++) {
            const uint8_t c = from.offset[j];
            if (c == '\n') {
                nl++;
                if (j == 0 || from.offset[j - 1] == '\n') bad = true;
            }
            if (c == 0) bad = nul = true;
        }
        horef[(size_t)i].nl = nl | (bad ? PPG_OFF_SERIAL : 0u) | (nul ? PPG_OFF_NUL : 0u);
        hoff.insert(hoff.end(), from.offset.begin(), from.offset.end());
    }
    HIPCHK(sh->dicts.alloc((size_t)n * kWin));
    ByteVec hwin;
    if (!windows_contig && n) {   // scattered windows: one staging copy, one H2D
        hwin.resize((size_t)n * kWin);
        for (int32_t i = 0; i < n; i++) memcpy(hwin.data() + (size_t)i * kWin, spec[i].window, kWin);
        windows_contig = hwin.data();
    }
    if (n) HIPCHK(hipMemcpyAsync(sh->dicts.p, windows_contig, (size_t)n * kWin, hipMemcpyHostToDevice, s));
    HIPCHK(sh->offs.alloc(hoff.size() + 16));
    if (!hoff.empty()) HIPCHK(hipMemcpyAsync(sh->offs.p, hoff.data(), hoff.size(), hipMemcpyHostToDevice, s));
    HIPCHK(sh->oref.alloc((size_t)n));
    HIPCHK(hipMemcpyAsync(sh->oref.p, horef.data(), sizeof(PpgOffsetRef) * (size_t)n, hipMemcpyHostToDevice, s));
    HIPCHK(sh->res.alloc((size_t)n));
    HIPCHK(sh->info.alloc((size_t)n));
    HIPCHK(sh->base.alloc((size_t)n));
    HIPCHK(sh->total.alloc(1));
    // output + a 64-byte tail: the parse kernels read whole 16-B words
    if ((size_t)out_cap + 64 > sh->out.n) HIPCHK(sh->out.alloc((size_t)out_cap + 64));
    sh->out_cap = (int64_t)sh->out.n - 64;
    HIPCHK(hipMemsetAsync(sh->out.p + out_cap, 0, 64, s));
    // descriptor space (16 B per record) for every record of the shard (all batches: copy_records
    // and the keys stay valid for multi-batch shards) sized for >= 256-B records; a batch that needs
    // more grows it, keeping the earlier batches' descriptors (batch_collect)
    HIPCHK(sh->recs.alloc((size_t)(4 * (total_out / 256 + 1024))));
    HIPCHK(sh->nls.alloc((size_t)nl_need + 64));
    if (!sh->ev[0])
        for (auto &e : sh->ev) HIPCHK(hipEventCreate(&e));
    if (!sh->h_tot) HIPCHK(hipHostMalloc((void **)&sh->h_tot, 8, hipHostMallocDefault));
    HIPCHK(hipStreamSynchronize(s));   // the host staging vectors above die here
    return PPG_OK;
}

// Size a shard's device buffers once for every range [first + a, first + b) it will be prepared for
// (with their side points when split), so that re-preparing it range after range never
// reallocates: a hipFree waits for the whole device, and in a pipeline of several shards (the
// cursor, host ingest) that stalled every other stream's decode and copies (r03: 300-560 ms per
// 8 GiB cursor batch).  shard_prepare / ppg_shard_set_split then find every buffer large enough.
int shard_reserve(ppg_shard *sh, const ppg_index *ix, int32_t first,
                  const std::vector<std::pair<int32_t, int32_t>> &ranges, bool split) {
    const auto &P = ix->pts;
    const auto &O = ix->side_out;
    int64_t n_max = 1, out_max = 0, off_max = 0, nsub_max = 0, nl_max = 0;
    uint64_t nl_bytes = kNlBytesPerEntry;
    if (const char *e = getenv("PPG_NL_BYTES")) nl_bytes = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    for (auto [a, b] : ranges) {
        const int64_t n = b - a, lo = P[(size_t)first + a].output, hi = P[(size_t)first + b].output;
        int64_t off = 0, nsub = 0;
        for (int32_t k = first + a; k < first + b; k++) off += (int64_t)P[(size_t)k].offset.size();
        if (split && !O.empty())
            nsub = (int64_t)(std::lower_bound(O.begin(), O.end(), hi) - std::upper_bound(O.begin(), O.end(), lo));
        nsub = std::max<int64_t>(nsub, 0);
        n_max = std::max(n_max, n);
        out_max = std::max(out_max, hi - lo);
        off_max = std::max(off_max, off);
        nsub_max = std::max(nsub_max, nsub);
        // census: the chunks' regions, then (split) the pieces' past them (ppg_shard_set_split)
        const int64_t per = nl_bytes >= (1ull << 40) ? 0 : (hi - lo) / (int64_t)nl_bytes;
        nl_max = std::max(nl_max, per + 64 * n + (nsub ? per + 64 * (n + nsub) : 0));
    }
    HIPCHK(sh->jobs.alloc((size_t)n_max));
    HIPCHK(sh->dicts.alloc((size_t)(n_max + nsub_max) * kWin));
    HIPCHK(sh->offs.alloc((size_t)off_max + 16));
    HIPCHK(sh->oref.alloc((size_t)n_max));
    HIPCHK(sh->res.alloc((size_t)n_max));
    HIPCHK(sh->info.alloc((size_t)n_max));
    HIPCHK(sh->base.alloc((size_t)n_max));
    HIPCHK(sh->total.alloc(1));
    HIPCHK(sh->out.alloc((size_t)out_max + 64));
    HIPCHK(sh->recs.alloc((size_t)(4 * (out_max / 256 + 1024))));
    HIPCHK(sh->nls.alloc((size_t)nl_max + 64));
    if (nsub_max) {
        HIPCHK(sh->sjobs.alloc((size_t)(n_max + nsub_max)));
        HIPCHK(sh->ljobs.alloc((size_t)(n_max + nsub_max)));
        HIPCHK(sh->linv.alloc((size_t)(n_max + nsub_max)));
        HIPCHK(sh->sres.alloc((size_t)(n_max + nsub_max)));
        HIPCHK(sh->sidx.alloc((size_t)n_max + 1));
    }
    return PPG_OK;
}

extern "C" {

int ppg_shard_create(ppg_ctx *ctx, const ppg_index *ix, int32_t first, int32_t n, const void *comp, int64_t comp_len,
                     int comp_on_device, int64_t out_capacity, ppg_shard **out) {
    if (!ctx || !ix || !comp || !out || n < 0 || first < 0 || (size_t)first + (size_t)n + 1 > ix->pts.size())
        return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(ctx->device));
    auto sh = std::unique_ptr<ppg_shard, void (*)(ppg_shard *)>(new ppg_shard, ppg_shard_free);
    sh->ctx = ctx;
    const uint8_t *dcomp = (const uint8_t *)comp;
    if (!comp_on_device) {
        hipStream_t s = ctx->stream;
        HIPCHK(sh->comp_own.alloc((size_t)comp_len + 64));
        HIPCHK(hipMemsetAsync(sh->comp_own.p + comp_len, 0, 64, s));
        HIPCHK(hipMemcpyAsync(sh->comp_own.p, comp, (size_t)comp_len, hipMemcpyHostToDevice, s));
        dcomp = sh->comp_own.p;
    }
    const int rc = shard_prepare(sh.get(), ix, first, n, dcomp, comp_len, out_capacity, ctx->stream);
    if (rc != PPG_OK) return rc;
    *out = sh.release();
    return PPG_OK;
}

}  // extern "C"

hipStream_t shard_stream(const ppg_shard *sh) { return sh->stream ? sh->stream : sh->ctx->stream; }

void shard_reset(ppg_shard *sh) {
    sh->t_inflate = sh->t_parse = sh->t_total = 0;
    sh->h_base.assign((size_t)sh->n, 0);
    sh->total_records = 0;
    sh->ran = 0;
}

// Enqueue one batch [b0, b1) on the shard's stream, with no host synchronisation: inflate (+ the
// fused newline census), per-chunk counts and their scan, the record total into pinned host
// memory, then the descriptors, whose writes stop at the descriptor buffer's size.
int batch_launch(ppg_shard *sh, int32_t b0, int32_t b1) {
    hipStream_t s = shard_stream(sh);
    const int nb = b1 - b0;
    HIPCHK(hipEventRecord(sh->ev[0], s));
    if (sh->nsub && sh->mat_n) {   // one batch: sub-jobs [0, mat_first) decoded, the rest materialised
        const uint32_t ns = sh->h_sidx[(size_t)sh->n];
        HIPCHK(ppg_launch_inflate(s, sh->ctx->ring_bits, sh->ctx->lit_bits, (const uint32_t *)sh->comp, sh->nwords,
                                  sh->ljobs.p, sh->dicts.p, sh->out.p, sh->sres.p, (int)sh->mat_first, sh->nls.p));
        HIPCHK(ppg_launch_materialize(s, sh->mat_sym, sh->mat_win, sh->mat_info, sh->ljobs.p + sh->mat_first, sh->out.p,
                                      sh->sres.p + sh->mat_first, (int)(ns - sh->mat_first), sh->nls.p));
        HIPCHK(ppg_launch_split_merge(s, sh->sjobs.p, sh->sres.p, sh->linv.p, sh->sidx.p + b0, sh->nls.p,
                                      sh->jobs.p + b0, sh->res.p + b0, sh->nls.p, nb));
    } else if (sh->nsub) {   // the batch's sub-jobs (longest first, see ppg_shard_set_split), then one result per chunk
        const uint32_t s0 = sh->h_sidx[(size_t)b0], s1 = sh->h_sidx[(size_t)b1];
        const bool lpt = sh->lpt;
        HIPCHK(ppg_launch_inflate(s, sh->ctx->ring_bits, sh->ctx->lit_bits, (const uint32_t *)sh->comp, sh->nwords,
                                  (lpt ? sh->ljobs.p : sh->sjobs.p) + s0, sh->dicts.p, sh->out.p, sh->sres.p + s0,
                                  (int)(s1 - s0), sh->nls.p));
        HIPCHK(ppg_launch_split_merge(s, sh->sjobs.p, sh->sres.p, lpt ? sh->linv.p : nullptr, sh->sidx.p + b0, sh->nls.p,
                                      sh->jobs.p + b0, sh->res.p + b0, sh->nls.p, nb));
    } else {
        HIPCHK(ppg_launch_inflate(s, sh->ctx->ring_bits, sh->ctx->lit_bits, (const uint32_t *)sh->comp, sh->nwords,
                                  sh->jobs.p + b0, sh->dicts.p, sh->out.p, sh->res.p + b0, nb, sh->nls.p));
    }
    HIPCHK(hipEventRecord(sh->ev[1], s));
    HIPCHK(ppg_launch_parse_count(s, sh->out.p, sh->jobs.p + b0, sh->res.p + b0, sh->offs.p, sh->oref.p + b0,
                                  sh->info.p + b0, sh->base.p + b0, sh->total.p, nb, sh->nls.p));
    HIPCHK(ppg_launch_total_to_host(s, sh->total.p, sh->h_tot));   // (a kernel store: no DMA engine, ppg_parse.hip)
    HIPCHK(hipEventRecord(sh->ev[2], s));
    // descriptors at the batch's shard-global record base (sh->total_records: batches of one shard
    // run one after the other), writes bounded by the buffer
    const uint64_t r0 = 4 * (uint64_t)sh->total_records;
    HIPCHK(ppg_launch_parse_emit(s, sh->out.p, sh->jobs.p + b0, sh->res.p + b0, sh->offs.p, sh->oref.p + b0,
                                 sh->info.p + b0, sh->base.p + b0, sh->nls.p, sh->recs.p + std::min<uint64_t>(r0, sh->recs.n),
                                 sh->recs.n > r0 ? (uint64_t)sh->recs.n - r0 : 0, nb));
    HIPCHK(hipEventRecord(sh->ev[3], s));
    return PPG_OK;
}

// Wait for a launched batch.  If its records did not fit the descriptor buffer (more than one
// record per 256 output bytes), grow the buffer and write the descriptors again.
int batch_collect(ppg_shard *sh, int32_t b0, int32_t b1, float &total_ms) {
    hipStream_t s = shard_stream(sh);
    const int nb = b1 - b0;
    HIPCHK(hipEventSynchronize(sh->ev[3]));
    const uint64_t tot = *sh->h_tot;
    float a = 0, b = 0, c = 0;
    HIPCHK(hipEventElapsedTime(&a, sh->ev[0], sh->ev[1]));
    HIPCHK(hipEventElapsedTime(&b, sh->ev[1], sh->ev[2]));   // counts + scan
    HIPCHK(hipEventElapsedTime(&c, sh->ev[2], sh->ev[3]));   // descriptors
    const uint64_t r0 = 4 * (uint64_t)sh->total_records;
    if ((size_t)(r0 + 4 * tot) > sh->recs.n) {
        // grow, keeping the earlier batches' descriptors, and write this batch's again
        DevBuf<uint32_t> grown;
        // half again what is needed: a shard whose records average under 256 B grows O(log) times,
        // not once per batch (each growth copies every earlier batch's descriptors)
        HIPCHK(grown.alloc((size_t)(r0 + 4 * tot + (r0 + 4 * tot) / 2 + 4096)));
        if (r0) HIPCHK(hipMemcpyAsync(grown.p, sh->recs.p, 4 * r0, hipMemcpyDeviceToDevice, s));
        std::swap(grown.p, sh->recs.p);
        std::swap(grown.n, sh->recs.n);
        HIPCHK(hipEventRecord(sh->ev[2], s));
        HIPCHK(ppg_launch_parse_emit(s, sh->out.p, sh->jobs.p + b0, sh->res.p + b0, sh->offs.p, sh->oref.p + b0,
                                     sh->info.p + b0, sh->base.p + b0, sh->nls.p, sh->recs.p + r0,
                                     (uint64_t)sh->recs.n - r0, nb));
        HIPCHK(hipEventRecord(sh->ev[3], s));
        HIPCHK(hipEventSynchronize(sh->ev[3]));
        float c2 = 0;
        HIPCHK(hipEventElapsedTime(&c2, sh->ev[2], sh->ev[3]));
        c += c2;
    }
    // spot keys of the batch's records while its output is resident (ppg_shard_set_keys); the next
    // batch's inflate follows on the same stream, so this output is read before it is overwritten
    if (sh->keys_dev) {
        if (sh->total_records + (int64_t)tot > sh->keys_cap) return PPG_BUF_ERROR;
        HIPCHK(ppg_launch_record_keys(s, sh->out.p, sh->jobs.p + b0, sh->res.p + b0, sh->offs.p, sh->oref.p + b0,
                                      sh->info.p + b0, sh->base.p + b0, sh->recs.p + r0,
                                      sh->keys_dev + sh->total_records, nb));
    }
    sh->t_inflate += a;
    sh->t_parse += b + c;
    total_ms += a + b + c;
    // batch-local bases -> shard-global
    std::vector<uint64_t> hb((size_t)nb);
    HIPCHK(hipMemcpyAsync(hb.data(), sh->base.p + b0, 8 * (size_t)nb, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < nb; i++) sh->h_base[(size_t)(b0 + i)] = (int64_t)hb[(size_t)i] + sh->total_records;
    sh->total_records += (int64_t)tot;
    return PPG_OK;
}

int shard_finish(ppg_shard *sh, float total_ms) {
    hipStream_t s = shard_stream(sh);
    sh->t_total = total_ms;
    sh->h_res.resize((size_t)sh->n);
    sh->h_info.resize((size_t)sh->n);
    if (sh->n) {
        HIPCHK(hipMemcpyAsync(sh->h_res.data(), sh->res.p, sizeof(PpgInflateResult) * (size_t)sh->n,
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(sh->h_info.data(), sh->info.p, sizeof(PpgParseInfo) * (size_t)sh->n,
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    sh->ran = 1;
    for (int32_t i = 0; i < sh->n; i++)
        if (sh->h_res[(size_t)i].status != 0) return sh->h_res[(size_t)i].status;
    return PPG_OK;
}

extern "C" {

static int shard_run(ppg_shard *sh) {
    HIPCHK(hipSetDevice(sh->ctx->device));
    shard_reset(sh);
    float total_ms = 0;
    for (auto [b0, b1] : sh->batches) {
        int rc = batch_launch(sh, b0, b1);
        if (rc == PPG_OK) rc = batch_collect(sh, b0, b1, total_ms);
        if (rc != PPG_OK) return rc;
    }
    return shard_finish(sh, total_ms);
}

int ppg_shard_run(ppg_shard *sh) {
    if (!sh) return PPG_ARG_ERROR;
    sh->keys_written = 0;
    sh->last_rc = shard_run(sh);
    sh->keys_written = sh->last_rc == PPG_OK && sh->keys_dev != nullptr;
    return sh->last_rc;
}

// Side points: deflate block starts strictly inside the shard's chunks (absolute file bit,
// absolute output offset, the 32 KiB of output before it).  Chunk k is then decoded by one wave
// per piece between its Point, its side points and the next Point; results are identical.
int ppg_shard_set_split(ppg_shard *sh, int32_t nsub, const int64_t *bit, const int64_t *output,
                        const uint8_t *windows) {
    if (!sh || nsub < 0 || (nsub && (!bit || !output || !windows))) return PPG_ARG_ERROR;
    return shard_set_split_impl(sh, nsub, bit, output, windows, true);
}

}  // extern "C"

// windows == nullptr: the pieces are not decoded from their side points (the lone-chunk Decompress
// materialises them from its pass-1 symbols, ppg_chunk.cpp): no dictionaries, no prev_byte; lpt =
// false: the caller sets the launch order (ljobs / linv) itself
int shard_set_split_impl(ppg_shard *sh, int32_t nsub, const int64_t *bit, const int64_t *output,
                         const uint8_t *windows, bool lpt) {
    HIPCHK(hipSetDevice(sh->ctx->device));
    hipStream_t s = shard_stream(sh);
    const int32_t n = sh->n;
    const std::vector<int64_t> &PO = sh->h_pout;
    const int64_t base_byte = sh->base_byte;
    // validate: sorted, strictly inside a chunk of the shard, bit inside that chunk's slice
    std::vector<uint32_t> hidx((size_t)n + 1, 0);
    {
        int32_t c = 0;
        for (int32_t t = 0; t < nsub; t++) {
            if (t && output[t] <= output[t - 1]) return PPG_ARG_ERROR;
            while (c < n && output[t] >= PO[(size_t)c + 1]) c++;
            if (c >= n || output[t] <= PO[(size_t)c]) return PPG_ARG_ERROR;
            const PpgInflateJob &J = sh->h_jobs[(size_t)c];
            const int64_t rb = bit[t] - 8 * base_byte;
            if (rb <= (int64_t)J.bit_start || rb >= (int64_t)J.bit_limit) return PPG_ARG_ERROR;
            hidx[(size_t)c + 1]++;
        }
    }
    sh->nsub = 0;
    sh->ran = 0;
    if (!nsub) return PPG_OK;
    for (int32_t k = 0; k < n; k++) hidx[(size_t)k + 1] += hidx[(size_t)k] + 1;   // + the chunk's own first piece
    uint64_t nl_bytes = kNlBytesPerEntry;
    if (const char *e = getenv("PPG_NL_BYTES")) nl_bytes = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    sh->h_sjobs.assign((size_t)n + (size_t)nsub, PpgInflateJob{});
    // census regions (batch-relative, like the chunks'): a chunk left whole keeps its own region of
    // sh->nls (nothing to merge); the pieces of a split chunk get regions past every chunk's of the
    // same batch, and the merge copies them back
    std::vector<uint64_t> nl_batch_end((size_t)n, 0);
    std::vector<uint8_t> batch_first((size_t)n, 0);
    uint64_t nl_need = 0;
    for (auto [b0, b1] : sh->batches) {
        uint64_t e = 0;
        for (int32_t k = b0; k < b1; k++)
            e = std::max<uint64_t>(e, sh->h_jobs[(size_t)k].nl_off + sh->h_jobs[(size_t)k].nl_cap);
        for (int32_t k = b0; k < b1; k++) nl_batch_end[(size_t)k] = e;
        if (b0 < b1) batch_first[(size_t)b0] = 1;
        nl_need = std::max(nl_need, e);
    }
    uint64_t nl_tot = 0;
    int32_t t = 0;
    for (int32_t k = 0; k < n; k++) {
        if (batch_first[(size_t)k]) nl_tot = nl_batch_end[(size_t)k];   // its pieces' regions: past its chunks'

        const PpgInflateJob &C = sh->h_jobs[(size_t)k];
        const int64_t from_out = PO[(size_t)k];
        if (hidx[(size_t)k + 1] - hidx[(size_t)k] == 1) {
            sh->h_sjobs[hidx[(size_t)k]] = C;
            continue;
        }
        for (uint32_t j = hidx[(size_t)k]; j < hidx[(size_t)k + 1]; j++) {
            PpgInflateJob J = C;
            int64_t lo = 0;   // chunk-relative start of this piece
            if (j > hidx[(size_t)k]) {
                const int32_t q = t++;
                lo = output[q] - from_out;
                J.bit_start = (uint64_t)(bit[q] - 8 * base_byte);
                J.dict_off = ((uint64_t)n + (uint64_t)q) * kWin;
                J.raw_shift = C.raw_shift + (uint32_t)lo;
                J.prev_byte = windows ? windows[(size_t)q * kWin + kWin - 1] : 0u;
            }
            const int64_t hi = j + 1 < hidx[(size_t)k + 1] ? output[t] - from_out : (int64_t)C.out_len;
            J.out_off = C.out_off + (uint64_t)lo;
            J.out_len = (uint64_t)(hi - lo);
            J.expect_end = ~0ull;
            const uint64_t cap = nl_bytes >= (1ull << 40) ? 0 : J.out_len / nl_bytes + 64;
            J.nl_off = nl_tot;
            J.nl_cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFFFu);
            nl_tot += J.nl_cap;
            nl_need = std::max(nl_need, nl_tot);
            sh->h_sjobs[j] = J;
        }
    }
    // dictionaries: the chunks' windows, then the side points' (in place when shard_reserve or an
    // earlier split left room)
    DevBuf<uint8_t> d2;
    if (windows && sh->dicts.n < ((size_t)n + (size_t)nsub) * kWin) {
        HIPCHK(d2.alloc(((size_t)n + (size_t)nsub) * kWin));
        HIPCHK(hipMemcpyAsync(d2.p, sh->dicts.p, (size_t)n * kWin, hipMemcpyDeviceToDevice, s));
        std::swap(sh->dicts.p, d2.p);
        std::swap(sh->dicts.n, d2.n);
    }
    if (windows)
        HIPCHK(hipMemcpyAsync(sh->dicts.p + (size_t)n * kWin, windows, (size_t)nsub * kWin, hipMemcpyHostToDevice, s));
    HIPCHK(sh->sjobs.alloc(sh->h_sjobs.size()));
    HIPCHK(hipMemcpyAsync(sh->sjobs.p, sh->h_sjobs.data(), sizeof(PpgInflateJob) * sh->h_sjobs.size(),
                          hipMemcpyHostToDevice, s));
    HIPCHK(sh->sres.alloc(sh->h_sjobs.size()));
    HIPCHK(sh->sidx.alloc(hidx.size()));
    HIPCHK(hipMemcpyAsync(sh->sidx.p, hidx.data(), 4 * hidx.size(), hipMemcpyHostToDevice, s));
    if ((size_t)nl_need + 64 > sh->nls.n) {   // grow, keeping nothing (the next run rewrites it)
        HIPCHK(sh->nls.alloc((size_t)nl_need + 64));
    }
    sh->h_sidx = hidx;
    // launch order: within each batch the sub-jobs longest first (LPT), so the launch drains on its
    // shortest pieces -- a chunk's pieces are whole deflate blocks of similar size, but the last one
    // before a Point, a pigz piece's flush block and a chunk left whole are not.  The results land
    // in launch order and ppg_split_merge reads them through the inverse permutation.
    // PPG_SPLIT_ORDER=0: the sub-jobs in chunk order.
    static const bool lpt_off = [] { const char *e = getenv("PPG_SPLIT_ORDER"); return e && *e == '0'; }();
    sh->lpt = lpt && !lpt_off;
    sh->mat_n = 0;
    if (sh->lpt) {
        const size_t ns = sh->h_sjobs.size();
        std::vector<uint32_t> perm(ns), inv(ns);
        std::vector<PpgInflateJob> lj(ns);
        for (auto [b0, b1] : sh->batches) {
            const uint32_t s0 = hidx[(size_t)b0], s1 = hidx[(size_t)b1];
            for (uint32_t j = s0; j < s1; j++) perm[j] = j;
            std::stable_sort(perm.begin() + s0, perm.begin() + s1, [&](uint32_t a, uint32_t b) {
                return sh->h_sjobs[a].out_len > sh->h_sjobs[b].out_len;
            });
        }
        for (size_t q = 0; q < ns; q++) {
            lj[q] = sh->h_sjobs[perm[q]];
            inv[perm[q]] = (uint32_t)q;
        }
        HIPCHK(sh->ljobs.alloc(ns));
        HIPCHK(sh->linv.alloc(ns));
        HIPCHK(hipMemcpyAsync(sh->ljobs.p, lj.data(), sizeof(PpgInflateJob) * ns, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(sh->linv.p, inv.data(), 4 * ns, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    HIPCHK(hipStreamSynchronize(s));   // staging vectors and d2 (the old dictionaries) die here
    sh->nsub = nsub;
    return PPG_OK;
}

extern "C" {

int ppg_shard_results(ppg_shard *sh, int64_t *records, int64_t *produced, int32_t *status, int32_t *flags,
                      int64_t *end_bit) {
    if (!sh || !sh->ran) return PPG_ARG_ERROR;
    for (int32_t i = 0; i < sh->n; i++) {
        const auto &r = sh->h_res[(size_t)i];
        if (records) records[i] = (int64_t)sh->h_info[(size_t)i].records;
        if (produced) produced[i] = (int64_t)r.produced;
        if (status) status[i] = r.status;
        if (flags) {
            int32_t f = r.flags;
            const auto &J = sh->h_jobs[(size_t)i];
            if (J.expect_end != ~0ull && r.status == 0 && r.end_bit != J.expect_end) f |= 4;   // end mismatch
            if (sh->h_info[(size_t)i].serial) f |= 8;                                         // serial parse
            flags[i] = f;
        }
        if (end_bit) end_bit[i] = (int64_t)r.end_bit;
    }
    return PPG_OK;
}

int64_t ppg_shard_total_records(ppg_shard *sh) { return sh && sh->ran ? sh->total_records : -1; }
int32_t ppg_shard_batches(ppg_shard *sh) { return sh ? (int32_t)sh->batches.size() : 0; }

int ppg_shard_copy_chunk(ppg_shard *sh, int32_t k, uint8_t *dst, int64_t cap, int64_t *len) {
    if (!sh || !sh->ran || sh->batches.size() != 1 || k < 0 || k >= sh->n || !dst) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(sh->ctx->device));
    const int64_t got = (int64_t)sh->h_res[(size_t)k].produced;
    if (got > cap) return PPG_BUF_ERROR;
    if (got) HIPCHK(hipMemcpy(dst, sh->out.p + sh->h_jobs[(size_t)k].out_off, (size_t)got, hipMemcpyDeviceToHost));
    if (len) *len = got;
    return PPG_OK;
}

int ppg_shard_copy_records(ppg_shard *sh, int32_t k, uint32_t *dst, int64_t cap, int64_t *nrec) {
    if (!sh || !sh->ran || k < 0 || k >= sh->n) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(sh->ctx->device));
    const int64_t r = (int64_t)sh->h_info[(size_t)k].records;
    if (nrec) *nrec = r;
    if (!dst) return PPG_OK;
    if (r > cap) return PPG_BUF_ERROR;
    if (r) HIPCHK(hipMemcpy(dst, sh->recs.p + 4 * sh->h_base[(size_t)k], 16 * (size_t)r, hipMemcpyDeviceToHost));
    return PPG_OK;
}

int ppg_shard_set_keys(ppg_shard *sh, int64_t *dev_keys, int64_t cap) {
    if (!sh || cap < 0 || (dev_keys == nullptr) != (cap == 0)) return PPG_ARG_ERROR;
    sh->keys_dev = dev_keys;
    sh->keys_cap = cap;
    sh->keys_written = 0;   // filled by the next run, not by an earlier one
    return PPG_OK;
}

int ppg_shard_keys_ready(ppg_shard *sh) { return sh && sh->keys_written ? 1 : 0; }

int ppg_shard_keys(ppg_shard *sh, int64_t *dev_keys, int64_t cap) {
    if (!sh || !sh->ran || sh->batches.size() != 1 || !dev_keys) return PPG_ARG_ERROR;
    if (cap < sh->total_records) return PPG_BUF_ERROR;
    HIPCHK(hipSetDevice(sh->ctx->device));
    hipStream_t s = sh->ctx->stream;
    HIPCHK(ppg_launch_record_keys(s, sh->out.p, sh->jobs.p, sh->res.p, sh->offs.p, sh->oref.p, sh->info.p, sh->base.p,
                                  sh->recs.p, dev_keys, sh->n));
    HIPCHK(hipStreamSynchronize(s));
    return PPG_OK;
}

int ppg_shard_record_base(ppg_shard *sh, int64_t *base) {
    if (!sh || !sh->ran || !base) return PPG_ARG_ERROR;
    std::copy(sh->h_base.begin(), sh->h_base.end(), base);
    return PPG_OK;
}

int ppg_shard_counts_to_device(ppg_shard *sh, int64_t *dev_dst) {
    if (!sh || !sh->ran || !dev_dst) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(sh->ctx->device));
    std::vector<int64_t> c((size_t)sh->n);
    for (int32_t i = 0; i < sh->n; i++) c[(size_t)i] = (int64_t)sh->h_info[(size_t)i].records;
    hipStream_t s = sh->ctx->stream;   // ordered after ppg_ctx_wait_stream
    if (sh->n) HIPCHK(hipMemcpyAsync(dev_dst, c.data(), 8 * (size_t)sh->n, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    return PPG_OK;
}

int ppg_shard_copy_output(ppg_shard *sh, int64_t off, int64_t len, void *dst, int dst_on_device) {
    if (!sh || !sh->ran || sh->batches.size() != 1 || off < 0 || len < 0 || (len && !dst)) return PPG_ARG_ERROR;
    const int64_t total = sh->h_pout[(size_t)sh->n] - sh->h_pout[0];
    if (off + len > total) return PPG_ARG_ERROR;
    if (!len) return PPG_OK;
    HIPCHK(hipSetDevice(sh->ctx->device));
    hipStream_t s = sh->ctx->stream;
    HIPCHK(hipMemcpyAsync(dst, sh->out.p + off, (size_t)len,
                          dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PPG_OK;
}

int ppg_shard_timing(ppg_shard *sh, float *inflate_ms, float *parse_ms, float *total_ms) {
    if (!sh || !sh->ran) return PPG_ARG_ERROR;
    if (inflate_ms) *inflate_ms = sh->t_inflate;
    if (parse_ms) *parse_ms = sh->t_parse;
    if (total_ms) *total_ms = sh->t_total;
    return PPG_OK;
}

// README "Decompress" (ppg_decompress_chunk): ppg_chunk.cpp

}  // extern "C"

// ================================ host ingest (file -> GPU) ================================
// pread [off, off+len) of fd into dst with `threads` parallel readers; false on a short read
bool pread_parallel(int fd, uint8_t *dst, int64_t off, int64_t len, int threads) {
    const int64_t part = std::max<int64_t>((len + threads - 1) / threads, 1 << 20);
    std::vector<std::thread> th;
    std::vector<int> ok;
    const int nparts = (int)std::max<int64_t>(1, (len + part - 1) / part);
    ok.assign((size_t)nparts, 1);
    for (int t = 0; t < nparts; t++) {
        th.emplace_back([=, &ok] {
            int64_t a = (int64_t)t * part, b = std::min(len, a + part);
            while (a < b) {
                const ssize_t r = pread(fd, dst + a, (size_t)(b - a), off + a);
                if (r <= 0) { ok[(size_t)t] = 0; return; }
                a += r;
            }
        });
    }
    for (auto &x : th) x.join();
    for (int v : ok) if (!v) return false;
    return true;
}

constexpr int kSlots = 16;    // pinned staging slots at most (IngestState::nslots are used)
constexpr int kPieces = 3;   // device piece slots: one finishing, one decoding, one filling

struct IngestState {
    // staging shape, fixed when the state is made: 4 slots of a quarter piece (<= 512 MiB) on one copy stream by default;
    // PPG_INGEST_SLOTS / PPG_INGEST_SLOT_MB / PPG_INGEST_COPY_STREAMS (1-2) for A/B runs (tools/ingest_probe.py)
    int nslots = 4, ncs = 1;
    int64_t slot_bytes = (int64_t)512 << 20;
    PinnedBuf slot[kSlots];       // pinned host staging, streamed through round-robin
    hipEvent_t slot_ev[kSlots] = {};
    hipStream_t cs2 = nullptr;    // a second copy stream (ncs == 2): odd slots
    hipEvent_t join_ev = nullptr; // cs2's copies of a piece, joined into cs before the piece's event
    DevBuf<uint8_t> db[kPieces];  // device copies of pieces
    hipStream_t cs = nullptr;     // copy stream
    hipStream_t ks[kPieces] = {};   // decode streams, one per piece slot
    hipEvent_t piece_ev[kPieces] = {};   // the piece's bytes are on the device (recorded on cs)
    ppg_shard *sh[kPieces] = {};
};

static void ingest_free(IngestState *st) {
    if (!st) return;
    for (int i = 0; i < kSlots; i++)
        if (st->slot_ev[i]) (void)hipEventDestroy(st->slot_ev[i]);
    if (st->join_ev) (void)hipEventDestroy(st->join_ev);
    if (st->cs2) (void)hipStreamDestroy(st->cs2);
    for (int i = 0; i < kPieces; i++) {
        if (st->sh[i]) ppg_shard_free(st->sh[i]);
        if (st->piece_ev[i]) (void)hipEventDestroy(st->piece_ev[i]);
    }
    if (st->cs) (void)hipStreamDestroy(st->cs);
    for (auto &k : st->ks) if (k) (void)hipStreamDestroy(k);
    delete st;
}

// the index's side points inside chunks [first, first+n) -> ppg_shard_set_split (host ingest)
int shard_split_from_index(ppg_shard *sh, const ppg_index *ix, int32_t first, int32_t n) {
    const int64_t lo = ix->pts[(size_t)first].output, hi = ix->pts[(size_t)first + n].output;
    const auto &O = ix->side_out;
    const size_t a = (size_t)(std::upper_bound(O.begin(), O.end(), lo) - O.begin());
    const size_t b = (size_t)(std::lower_bound(O.begin(), O.end(), hi) - O.begin());
    if (b <= a) return PPG_OK;
    return ppg_shard_set_split(sh, (int32_t)(b - a), ix->side_bit.data() + a, O.data() + a,
                               ix->side_win.data() + a * kWin);
}

extern "C" {

int ppg_file_release(ppg_ctx *ctx) {
    if (!ctx) return PPG_ARG_ERROR;
    if (ctx->ingest) {
        HIPCHK(hipSetDevice(ctx->device));
        ingest_free(ctx->ingest);
        ctx->ingest = nullptr;
    }
    return PPG_OK;
}

int ppg_file_decompress_all(ppg_ctx *ctx, const ppg_index *ix, const char *gz_path, int32_t first, int32_t n,
                            int64_t piece_bytes, int threads, int64_t *records, int64_t *total_records,
                            double *seconds) {
    if (!ctx || !ix || !gz_path || n < 0 || first < 0 || (size_t)first + (size_t)n + 1 > ix->pts.size())
        return PPG_ARG_ERROR;
    const auto &P = ix->pts;
    if (piece_bytes <= 0) piece_bytes = (int64_t)8 << 30;   // ~8k chunks at chunk=10000: one full wave generation
    if (threads <= 0) threads = 8;
    const bool verbose = getenv("PPG_INGEST_VERBOSE") != nullptr;
    HIPCHK(hipSetDevice(ctx->device));
    const auto t0 = std::chrono::steady_clock::now();
    auto now_ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const int fd = open(gz_path, O_RDONLY);
    if (fd < 0) return PPG_IO_ERROR;
    struct FdClose { int fd; ~FdClose() { close(fd); } } fdc{fd};

    // an index with side points (ppg_index_build_gpu_side) splits chunks when the file has too few
    // of them to fill the GPU a few times over (the ~6 generations bench.py's auto split uses)
    bool split = false;
    if (!ix->side_out.empty()) {
        int cus = 0;
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
        split = (int64_t)n < 6 * 32 * (int64_t)cus;
    }

    // pieces: consecutive chunks of about piece_bytes compressed bytes (at least one chunk).
    // (Ramping the first / last pieces down measured slower: one chunk alone takes ~100 ms, so
    // small pieces neither start nor drain the GPU faster; r06, with the last pieces split at side
    // points: 1.45-1.50 vs 1.34-1.36 s, 1.10 vs 1.09 s per 50 GB member, tools/ingest_probe.py.)
    std::vector<std::pair<int32_t, int32_t>> pieces;
    int64_t maxlen = 0;
    for (int32_t a = 0; a < n;) {
        int32_t b = a + 1;
        while (b < n && P[(size_t)first + b + 1].input - P[(size_t)first + a].input + 1 <= piece_bytes) b++;
        pieces.push_back({a, b});
        maxlen = std::max(maxlen, P[(size_t)first + b].input - P[(size_t)first + a].input + 1);
        a = b;
    }
    auto range = [&](size_t k, int64_t &off, int64_t &len) {
        off = P[(size_t)first + pieces[k].first].input - 1;
        len = P[(size_t)first + pieces[k].second].input - P[(size_t)first + pieces[k].first].input + 1;
    };

    // buffers persist in the ctx across calls (pinning and device allocation are slow)
    if (!ctx->ingest) {
        auto st = new IngestState;
        ctx->ingest = st;
        auto env_int = [](const char *k, int64_t d, int64_t lo, int64_t hi) {
            const char *e = getenv(k);
            return e ? std::min(hi, std::max(lo, (int64_t)strtoll(e, nullptr, 10))) : d;
        };
        st->nslots = (int)env_int("PPG_INGEST_SLOTS", 4, 2, kSlots);
        // slots of a quarter piece, at most 512 MiB (r06: 4 x 512 MiB vs 4 x 128 MiB pinned slots,
        // 1.02-1.05 vs 1.16-1.24 s per 50 GB member in one process: fewer, longer preads and copies;
        // 1 GiB slots no better -- profiles/r06v_ingest_slots.json); sized by the first call
        const int64_t auto_mb = std::min<int64_t>(512, std::max<int64_t>(8, (maxlen / 4 + (1 << 20) - 1) >> 20));
        st->slot_bytes = env_int("PPG_INGEST_SLOT_MB", auto_mb, 8, 1024) << 20;
        st->ncs = (int)env_int("PPG_INGEST_COPY_STREAMS", 1, 1, 2);
        // the copy stream at the greatest priority, i.e. on a hardware queue of its own: a stream
        // sharing a queue with a decode stream runs in order behind its kernels, and the piece copies
        // then wait for a whole decode (r06: one ~131 ms stall per 50 GB ingest whenever the runtime,
        // GPU_MAX_HW_QUEUES = 4, mapped the copy stream onto a piece stream's queue; gone at the
        // greatest priority or with 8 queues -- tools/ingest_probe.py).  PPG_INGEST_COPY_PRIO=0: off.
        if (env_int("PPG_INGEST_COPY_PRIO", 1, 0, 1)) {
            int lo = 0, hi = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHK(hipStreamCreateWithPriority(&st->cs, hipStreamNonBlocking, hi));
        } else {
            HIPCHK(hipStreamCreateWithFlags(&st->cs, hipStreamNonBlocking));
        }
        if (st->ncs == 2) {
            HIPCHK(hipStreamCreateWithFlags(&st->cs2, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&st->join_ev, hipEventDisableTiming));
        }
        for (int i = 0; i < st->nslots; i++) {
            HIPCHK(hipEventCreateWithFlags(&st->slot_ev[i], hipEventDisableTiming));
            HIPCHK(st->slot[i].alloc((size_t)st->slot_bytes));
        }
        for (int i = 0; i < kPieces; i++) {
            st->sh[i] = new ppg_shard;
            st->sh[i]->ctx = ctx;
            HIPCHK(hipStreamCreateWithFlags(&st->ks[i], hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&st->piece_ev[i], hipEventDisableTiming));
            st->sh[i]->stream = st->ks[i];
        }
    }
    IngestState &S = *ctx->ingest;
    for (int i = 0; i < kPieces; i++) {
        HIPCHK(S.db[i].alloc((size_t)maxlen + 64));
        if (int r = shard_reserve(S.sh[i], ix, first, pieces, split)) return r;
    }
    if (verbose) fprintf(stderr, "[ingest] %zu pieces, max %.1f MB, setup %.1f ms\n", pieces.size(), maxlen / 1e6, now_ms());

    // Producer thread: piece k -> device buffer k % kPieces (pread into pinned slots, H2D on the
    // copy stream, slot by slot), an event when its bytes are there.  Consumer (this thread): piece
    // k's jobs / windows / offsets (shard_prepare, on the piece's decode stream, which waits for that
    // event on the device), then its launch -- so a piece's prepare (~14 ms at 8 GiB: 9k windows
    // staged and copied) overlaps the next piece's read instead of delaying it (r05).
    const size_t np = pieces.size();
    std::mutex mu;
    std::condition_variable cv;
    size_t ready = 0, done = 0;
    int prod_rc = PPG_OK;
    bool stop = false;
    auto producer = [&] {
        (void)hipSetDevice(ctx->device);
        int rcp = PPG_OK;
        size_t slot = 0;
        for (size_t k = 0; k < np && rcp == PPG_OK; k++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || k < done + kPieces; });
                if (stop) return;
            }
            const double t1 = now_ms();
            int64_t off, len;
            range(k, off, len);
            uint8_t *dst = S.db[k % kPieces].p;
            double wait_ms = 0, read_ms = 0, slow_ms = 0, enq_ms = 0;   // (PPG_INGEST_VERBOSE) slot waits, preads, slowest pread, copy enqueues
            for (int64_t r = 0; r < len && rcp == PPG_OK; r += S.slot_bytes, slot = (slot + 1) % S.nslots) {
                const int64_t m = std::min(S.slot_bytes, len - r);
                hipStream_t cs = S.ncs == 2 && (slot & 1) ? S.cs2 : S.cs;
                const double tw = verbose ? now_ms() : 0;
                if (hipEventSynchronize(S.slot_ev[slot]) != hipSuccess) { rcp = PPG_DEVICE_ERROR; break; }
                const double tr = verbose ? now_ms() : 0;
                if (!pread_parallel(fd, S.slot[slot].p, off + r, m, threads)) { rcp = PPG_IO_ERROR; break; }
                if (verbose) {
                    const double te = now_ms();
                    wait_ms += tr - tw;
                    read_ms += te - tr;
                    slow_ms = std::max(slow_ms, te - tr);
                }
                const double tq = verbose ? now_ms() : 0;
                if (hipMemcpyAsync(dst + r, S.slot[slot].p, (size_t)m, hipMemcpyHostToDevice, cs) != hipSuccess ||
                    hipEventRecord(S.slot_ev[slot], cs) != hipSuccess)
                    rcp = PPG_DEVICE_ERROR;
                if (verbose) {
                    const double dq = now_ms() - tq;
                    enq_ms += dq;
                    if (dq > 5) fprintf(stderr, "[ingest] piece %zu: a copy's enqueue took %.1f ms at %.1f ms\n", k, dq, tq);
                    if (tr - tw > 20) fprintf(stderr, "[ingest] piece %zu: slot %zu waited %.1f ms at %.1f ms\n", k, slot, tr - tw, tw);
                }
            }
            if (rcp == PPG_OK && S.ncs == 2 &&
                (hipEventRecord(S.join_ev, S.cs2) != hipSuccess || hipStreamWaitEvent(S.cs, S.join_ev, 0) != hipSuccess))
                rcp = PPG_DEVICE_ERROR;
            if (rcp == PPG_OK && (hipMemsetAsync(dst + len, 0, 64, S.cs) != hipSuccess ||
                                  hipEventRecord(S.piece_ev[k % kPieces], S.cs) != hipSuccess))
                rcp = PPG_DEVICE_ERROR;
            if (verbose)
                fprintf(stderr, "[ingest] piece %zu: %.1f MB read+copy at %.1f ms in %.1f ms (pread %.1f ms, slowest "
                        "slot %.1f ms; waiting for pinned slots %.1f ms; copy enqueues %.1f ms)\n", k, len / 1e6, t1,
                        now_ms() - t1, read_ms, slow_ms, wait_ms, enq_ms);
            std::lock_guard<std::mutex> lk(mu);
            if (rcp != PPG_OK) prod_rc = rcp;
            else ready = k + 1;
            cv.notify_all();
        }
    };
    std::thread prod(producer);
    struct Joiner {
        std::thread &t; std::mutex &m; std::condition_variable &c; bool &stop;
        ~Joiner() { { std::lock_guard<std::mutex> lk(m); stop = true; } c.notify_all(); if (t.joinable()) t.join(); }
    } joiner{prod, mu, cv, stop};

    // Consumer: piece k is launched on its own stream as soon as it is ready, and only then is
    // piece k-1 collected, so piece k's waves fill the CUs that piece k-1's last waves leave idle
    // (a piece is ~1.1 generations of resident waves: its tail would otherwise idle the GPU).
    int64_t total = 0;
    int rc = PPG_OK;
    auto collect = [&](size_t k) -> int {
        ppg_shard *sh = S.sh[k % kPieces];
        float ms = 0;
        const double tc = now_ms();
        int r = batch_collect(sh, 0, sh->n, ms);
        const double tc1 = now_ms();
        if (r == PPG_OK) r = shard_finish(sh, ms);
        if (verbose)
            fprintf(stderr, "[ingest] piece %zu: collect from %.1f ms: batch_collect %.1f ms, finish %.1f ms\n", k, tc,
                    tc1 - tc, now_ms() - tc1);
        const int32_t a = pieces[k].first, b = pieces[k].second;
        if (verbose)
            fprintf(stderr, "[ingest] piece %zu: %d chunks collected at %.1f ms (kernels %.1f)\n", k, b - a, now_ms(),
                    sh->t_total);
        if (sh->ran) {
            for (int32_t i = 0; i < b - a; i++) {
                const int64_t r2 = (int64_t)sh->h_info[(size_t)i].records;
                if (records) records[a + i] = r2;
                total += r2;
            }
        }
        std::lock_guard<std::mutex> lk(mu);
        done = k + 1;
        cv.notify_all();
        return r;
    };
    for (size_t k = 0; k < np; k++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return ready > k || prod_rc != PPG_OK; });
            if (ready <= k) { rc = prod_rc; break; }
        }
        ppg_shard *sh = S.sh[k % kPieces];
        const double tp = now_ms();
        int64_t off, len;
        range(k, off, len);
        if (hipStreamWaitEvent(S.ks[k % kPieces], S.piece_ev[k % kPieces], 0) != hipSuccess) { rc = PPG_DEVICE_ERROR; break; }
        rc = shard_prepare(sh, ix, first + pieces[k].first, pieces[k].second - pieces[k].first, S.db[k % kPieces].p, len,
                           0, S.ks[k % kPieces]);
        const double tp1 = now_ms();
        if (rc == PPG_OK && split)
            rc = shard_split_from_index(sh, ix, first + pieces[k].first, pieces[k].second - pieces[k].first);
        if (rc != PPG_OK) break;
        const double tp2 = now_ms();
        shard_reset(sh);
        rc = sh->batches.size() == 1 ? batch_launch(sh, 0, sh->n) : PPG_ARG_ERROR;
        if (verbose)
            fprintf(stderr, "[ingest] piece %zu: prepared in %.1f ms (prepare %.1f, split %.1f, launch %.1f), launched at "
                    "%.1f ms\n", k, now_ms() - tp, tp1 - tp, tp2 - tp1, now_ms() - tp2, now_ms());
        if (rc != PPG_OK) break;
        if (k > 0 && (rc = collect(k - 1)) != PPG_OK) break;
    }
    if (rc == PPG_OK && np > 0) rc = collect(np - 1);
    hipStream_t cs = S.cs;
    HIPCHK(hipStreamSynchronize(cs));
    if (S.cs2) HIPCHK(hipStreamSynchronize(S.cs2));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (total_records) *total_records = total;
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

}  // extern "C"

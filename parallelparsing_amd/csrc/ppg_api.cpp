// ppg_api.cpp — host side of libppgpu.so: the C ABI declared in include/ppgpu.h.
//
//   Index model + CreateIndex      Common/Index.cs, Decompressor/Core.cs:14-131 (serial zlib pass)
//   .gzi Serialize / Deserialize   Common/IndexIO.cs:7-53
//   ppg_ctx                        one GPU, one HIP stream
//   ppg_shard                      DecompressAll over chunks [first, first+n): device-resident
//                                  compressed range + windows + offsets, batched inflate + parse
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

#include "../../include/ppgpu.h"
#include "ppg_device.h"

// launchers (ppg_inflate.hip, ppg_parse.hip)
size_t ppg_inflate_lds_bytes(int ring_bits, int lit_bits);
hipError_t ppg_launch_inflate(hipStream_t s, int ring_bits, int lit_bits, const uint32_t *comp, uint64_t nwords,
                              const PpgInflateJob *jobs, const uint8_t *dicts, uint8_t *out, PpgInflateResult *res,
                              int njobs);
hipError_t ppg_launch_parse_count(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  PpgParseInfo *info, uint64_t *base, uint64_t *total, int n);
hipError_t ppg_launch_parse_emit(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                 const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                 PpgParseInfo *info, const uint64_t *base, uint32_t *recs, int n);

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
constexpr int kChunk = PPG_CHUNK;
}

// ====================================== Index ======================================
struct PpgPoint {                       // Common/Index.cs:51-82
    int64_t output = 0;                 // offset in the uncompressed stream
    int64_t input = 0;                  // offset of the first full byte in the .gz
    int32_t bits = 0;                   // unused bits (1-7) of byte input-1, or 0
    std::vector<uint8_t> window;        // the preceding 32 KiB of output, oldest first
    std::vector<uint8_t> offset;        // bytes since the last '@' (the partial record)
};

struct ppg_index {
    int32_t chunk_max_bytes = 0;
    std::vector<PpgPoint> pts;

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
        p.window.resize(kWin);
        // oldest bytes (those after the circular write head) first
        std::copy(circ + (kWin - left), circ + kWin, p.window.begin());
        std::copy(circ, circ + (kWin - left), p.window.begin() + left);
        p.offset.assign(off, off + off_len);
        pts.push_back(std::move(p));
    }
};

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
    for (const auto &p : ix->pts) {
        const int32_t wl = (int32_t)p.window.size(), ol = (int32_t)p.offset.size();
        ok &= write_all(f, &p.output, 8) && write_all(f, &p.input, 8) && write_all(f, &p.bits, 4);
        ok &= write_all(f, &wl, 4) && write_all(f, p.window.data(), p.window.size());
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
    for (int32_t i = 0; ok && i < hdr[2]; i++) {
        PpgPoint p;
        int32_t wl = 0, ol = 0;
        ok = read_all(f, &p.output, 8) && read_all(f, &p.input, 8) && read_all(f, &p.bits, 4) && read_all(f, &wl, 4) &&
             wl >= 0;
        if (!ok) break;
        p.window.resize((size_t)wl);
        ok = read_all(f, p.window.data(), (size_t)wl) && read_all(f, &ol, 4) && ol >= 0;
        if (!ok) break;
        p.offset.resize((size_t)ol);
        ok = read_all(f, p.offset.data(), (size_t)ol);
        if (wl < kWin) p.window.resize(kWin, 0);
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
    size_t o = 0;
    for (int32_t i = 0; i < count; i++) {
        PpgPoint &p = ix->pts[(size_t)i];
        p.output = output[i];
        p.input = input[i];
        p.bits = bits[i];
        p.window.assign(windows + (size_t)i * kWin, windows + (size_t)(i + 1) * kWin);
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
    return ix->pts[(size_t)i].window.data();
}

const uint8_t *ppg_index_offset(const ppg_index *ix, int32_t i) {
    if (!ix || i < 0 || (size_t)i >= ix->pts.size()) return nullptr;
    return ix->pts[(size_t)i].offset.data();
}

void ppg_index_free(ppg_index *ix) { delete ix; }

const char *ppg_version(void) { return "ppgpu 0.1 gfx950 (wave-per-chunk inflate, LDS 32 KiB ring)"; }

}  // extern "C"

// ====================================== device ======================================
struct ppg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int ring_bits = 10;   // inflate history ring: 2^10..2^15 bytes of LDS per wavefront (1 KiB: 32 waves/CU)
    int lit_bits = 8;     // litlen root table: 2^8 entries (codes <= 8 bits: 99.65% of FASTQ tokens)
};

namespace {

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
    if (const char *rb = getenv("PPG_RING_BITS")) ctx->ring_bits = std::min(15, std::max(10, atoi(rb)));
    if (const char *lb = getenv("PPG_LIT_BITS")) ctx->lit_bits = std::min(9, std::max(8, atoi(lb)));
    if (ppg_inflate_lds_bytes(ctx->ring_bits, ctx->lit_bits) == 0) { ctx->ring_bits = 10; ctx->lit_bits = 8; }
    *out = ctx.release();
    return PPG_OK;
}

void ppg_close(ppg_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void *ppg_ctx_stream(ppg_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

}  // extern "C"

// ====================================== shard ======================================
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
    DevBuf<uint32_t> recs;
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
    int ran = 0;
};

extern "C" {

void ppg_shard_free(ppg_shard *sh) {
    if (!sh) return;
    (void)hipSetDevice(sh->ctx->device);
    for (auto &e : sh->ev) if (e) (void)hipEventDestroy(e);
    delete sh;
}

int ppg_shard_create(ppg_ctx *ctx, const ppg_index *ix, int32_t first, int32_t n, const void *comp, int64_t comp_len,
                     int comp_on_device, int64_t out_capacity, ppg_shard **out) {
    if (!ctx || !ix || !comp || !out || n < 0 || first < 0 || (size_t)first + (size_t)n + 1 > ix->pts.size())
        return PPG_ARG_ERROR;
    const auto &P = ix->pts;
    const int64_t base_byte = P[(size_t)first].input - 1;
    if (base_byte < 0) return PPG_ARG_ERROR;
    if (comp_len != P[(size_t)first + n].input - P[(size_t)first].input + 1) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(ctx->device));
    auto sh = std::unique_ptr<ppg_shard, void (*)(ppg_shard *)>(new ppg_shard, ppg_shard_free);
    sh->ctx = ctx;
    sh->first = first;
    sh->n = n;
    sh->comp_len = comp_len;
    sh->nwords = (uint64_t)(comp_len + 3) / 4;
    hipStream_t s = ctx->stream;
    if (comp_on_device) {
        if (((uintptr_t)comp & 3) != 0) return PPG_ARG_ERROR;
        sh->comp = (const uint8_t *)comp;
    } else {
        HIPCHK(sh->comp_own.alloc((size_t)comp_len + 64));
        HIPCHK(hipMemsetAsync(sh->comp_own.p + comp_len, 0, 64, s));
        HIPCHK(hipMemcpyAsync(sh->comp_own.p, comp, (size_t)comp_len, hipMemcpyHostToDevice, s));
        sh->comp = sh->comp_own.p;
    }
    // batches: consecutive chunks whose outputs fit out_capacity (0 = everything at once)
    int64_t total_out = P[(size_t)first + n].output - P[(size_t)first].output;
    if (total_out < 0) return PPG_ARG_ERROR;
    int64_t cap = out_capacity > 0 ? out_capacity : total_out;
    sh->h_jobs.resize((size_t)n);
    {
        int32_t b0 = 0;
        int64_t bbase = P[(size_t)first].output;
        int64_t need_max = 0;
        for (int32_t i = 0; i < n; i++) {
            const PpgPoint &from = P[(size_t)first + i], &to = P[(size_t)first + i + 1];
            int64_t ulen = to.output - from.output;
            if (ulen < 0) ulen = 0;   // Core.cs:145: len < 0 -> nothing produced
            if (to.output - bbase > cap && i > b0) {
                sh->batches.push_back({b0, i});
                need_max = std::max(need_max, from.output - bbase);
                b0 = i;
                bbase = from.output;
            }
            PpgInflateJob &J = sh->h_jobs[(size_t)i];
            J.bit_start = (uint64_t)(8 * (from.input - base_byte) - from.bits);
            J.bit_limit = (uint64_t)(8 * (to.input - base_byte));
            J.out_off = (uint64_t)(from.output - bbase);
            J.out_len = (uint64_t)ulen;
            J.dict_off = (uint64_t)i * kWin;
            J.expect_end = (size_t)first + i + 2 == P.size() ? ~0ull : (uint64_t)(8 * (to.input - base_byte) - to.bits);
        }
        if (n > 0) {
            sh->batches.push_back({b0, n});
            need_max = std::max(need_max, P[(size_t)first + n].output - bbase);
        }
        sh->out_cap = std::max<int64_t>(need_max, 0);
    }
    HIPCHK(sh->jobs.alloc((size_t)n));
    HIPCHK(hipMemcpyAsync(sh->jobs.p, sh->h_jobs.data(), sizeof(PpgInflateJob) * (size_t)n, hipMemcpyHostToDevice, s));
    // windows and offsets of the shard's `from` points
    std::vector<uint8_t> hwin((size_t)n * kWin);
    std::vector<PpgOffsetRef> horef((size_t)n);
    std::vector<uint8_t> hoff;
    for (int32_t i = 0; i < n; i++) {
        const PpgPoint &from = P[(size_t)first + i];
        if (from.window.size() < (size_t)kWin) return PPG_ARG_ERROR;
        memcpy(hwin.data() + (size_t)i * kWin, from.window.data(), kWin);
        horef[(size_t)i].start = hoff.size();
        horef[(size_t)i].len = (uint32_t)from.offset.size();
        hoff.insert(hoff.end(), from.offset.begin(), from.offset.end());
    }
    HIPCHK(sh->dicts.alloc(hwin.size()));
    HIPCHK(hipMemcpyAsync(sh->dicts.p, hwin.data(), hwin.size(), hipMemcpyHostToDevice, s));
    HIPCHK(sh->offs.alloc(hoff.size() + 16));
    if (!hoff.empty()) HIPCHK(hipMemcpyAsync(sh->offs.p, hoff.data(), hoff.size(), hipMemcpyHostToDevice, s));
    HIPCHK(sh->oref.alloc((size_t)n));
    HIPCHK(hipMemcpyAsync(sh->oref.p, horef.data(), sizeof(PpgOffsetRef) * (size_t)n, hipMemcpyHostToDevice, s));
    HIPCHK(sh->res.alloc((size_t)n));
    HIPCHK(sh->info.alloc((size_t)n));
    HIPCHK(sh->base.alloc((size_t)n));
    HIPCHK(sh->total.alloc(1));
    // output + a 64-byte tail: the parse kernels read whole 16-B words
    HIPCHK(sh->out.alloc((size_t)sh->out_cap + 64));
    HIPCHK(hipMemsetAsync(sh->out.p + sh->out_cap, 0, 64, s));
    // descriptor space (16 B per record) sized for >= 256-B records; a batch that needs more
    // grows it before its emit pass (ppg_shard_run)
    HIPCHK(sh->recs.alloc((size_t)(4 * (sh->out_cap / 256 + 1024))));
    for (auto &e : sh->ev) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipStreamSynchronize(s));
    *out = sh.release();
    return PPG_OK;
}

int ppg_shard_run(ppg_shard *sh) {
    if (!sh) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(sh->ctx->device));
    hipStream_t s = sh->ctx->stream;
    sh->t_inflate = sh->t_parse = sh->t_total = 0;
    sh->h_base.assign((size_t)sh->n, 0);
    sh->total_records = 0;
    float total_ms = 0;
    for (auto [b0, b1] : sh->batches) {
        const int nb = b1 - b0;
        HIPCHK(hipEventRecord(sh->ev[0], s));
        HIPCHK(ppg_launch_inflate(s, sh->ctx->ring_bits, sh->ctx->lit_bits, (const uint32_t *)sh->comp, sh->nwords, sh->jobs.p + b0,
                                  sh->dicts.p, sh->out.p, sh->res.p + b0, nb));
        HIPCHK(hipEventRecord(sh->ev[1], s));
        HIPCHK(ppg_launch_parse_count(s, sh->out.p, sh->jobs.p + b0, sh->res.p + b0, sh->offs.p, sh->oref.p + b0,
                                      sh->info.p + b0, sh->base.p + b0, sh->total.p, nb));
        uint64_t tot = 0;
        HIPCHK(hipMemcpyAsync(&tot, sh->total.p, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if ((size_t)(4 * tot) > sh->recs.n) HIPCHK(sh->recs.alloc((size_t)(4 * tot + 4096)));
        HIPCHK(hipEventRecord(sh->ev[2], s));
        HIPCHK(ppg_launch_parse_emit(s, sh->out.p, sh->jobs.p + b0, sh->res.p + b0, sh->offs.p, sh->oref.p + b0,
                                     sh->info.p + b0, sh->base.p + b0, sh->recs.p, nb));
        HIPCHK(hipEventRecord(sh->ev[3], s));
        HIPCHK(hipEventSynchronize(sh->ev[3]));
        float a = 0, b = 0, c = 0;
        HIPCHK(hipEventElapsedTime(&a, sh->ev[0], sh->ev[1]));
        HIPCHK(hipEventElapsedTime(&b, sh->ev[1], sh->ev[2]));   // count + scan (+ host read of the total)
        HIPCHK(hipEventElapsedTime(&c, sh->ev[2], sh->ev[3]));
        sh->t_inflate += a;
        sh->t_parse += b + c;
        total_ms += a + b + c;
        // batch-local bases -> shard-global
        std::vector<uint64_t> hb((size_t)nb);
        HIPCHK(hipMemcpy(hb.data(), sh->base.p + b0, 8 * (size_t)nb, hipMemcpyDeviceToHost));
        for (int i = 0; i < nb; i++) sh->h_base[(size_t)(b0 + i)] = (int64_t)hb[(size_t)i] + sh->total_records;
        sh->total_records += (int64_t)tot;
    }
    sh->t_total = total_ms;
    sh->h_res.resize((size_t)sh->n);
    sh->h_info.resize((size_t)sh->n);
    if (sh->n) {
        HIPCHK(hipMemcpy(sh->h_res.data(), sh->res.p, sizeof(PpgInflateResult) * (size_t)sh->n, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(sh->h_info.data(), sh->info.p, sizeof(PpgParseInfo) * (size_t)sh->n, hipMemcpyDeviceToHost));
    }
    sh->ran = 1;
    for (int32_t i = 0; i < sh->n; i++)
        if (sh->h_res[(size_t)i].status != 0) return sh->h_res[(size_t)i].status;
    return PPG_OK;
}

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
    if (!sh || !sh->ran || sh->batches.size() != 1 || k < 0 || k >= sh->n) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(sh->ctx->device));
    const int64_t r = (int64_t)sh->h_info[(size_t)k].records;
    if (nrec) *nrec = r;
    if (!dst) return PPG_OK;
    if (r > cap) return PPG_BUF_ERROR;
    if (r) HIPCHK(hipMemcpy(dst, sh->recs.p + 4 * sh->h_base[(size_t)k], 16 * (size_t)r, hipMemcpyDeviceToHost));
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
    if (sh->n) HIPCHK(hipMemcpy(dev_dst, c.data(), 8 * (size_t)sh->n, hipMemcpyHostToDevice));
    return PPG_OK;
}

int ppg_shard_timing(ppg_shard *sh, float *inflate_ms, float *parse_ms, float *total_ms) {
    if (!sh || !sh->ran) return PPG_ARG_ERROR;
    if (inflate_ms) *inflate_ms = sh->t_inflate;
    if (parse_ms) *parse_ms = sh->t_parse;
    if (total_ms) *total_ms = sh->t_total;
    return PPG_OK;
}

// README "Decompress": one checkpoint from a host slice, through a one-chunk shard.
int ppg_decompress_chunk(ppg_ctx *ctx, const ppg_index *ix, int32_t k, const uint8_t *slice, int64_t slice_len,
                         uint8_t *out, int64_t out_cap, int64_t *produced, uint32_t *recs, int64_t rec_cap,
                         int64_t *nrec) {
    if (!ctx || !ix || !slice || k < 0 || (size_t)k + 1 >= ix->pts.size()) return PPG_ARG_ERROR;
    ppg_shard *sh = nullptr;
    int rc = ppg_shard_create(ctx, ix, k, 1, slice, slice_len, 0, 0, &sh);
    if (rc != PPG_OK) return rc;
    rc = ppg_shard_run(sh);
    if (rc == PPG_OK) {
        int64_t len = 0;
        if (out) rc = ppg_shard_copy_chunk(sh, 0, out, out_cap, &len);
        else len = (int64_t)sh->h_res[0].produced;
        if (produced) *produced = len;
        if (rc == PPG_OK) rc = ppg_shard_copy_records(sh, 0, recs, rec_cap, nrec);
    }
    ppg_shard_free(sh);
    return rc;
}

}  // extern "C"

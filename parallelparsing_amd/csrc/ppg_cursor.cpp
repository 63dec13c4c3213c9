// ppg_cursor.cpp — bounded-memory record streaming of DecompressAll through the C ABI.
//
// The reference's BatchedFASTQ (Decompressor/BatchedFASTQ.cs:29-101) hands out records from a
// bounded cache (RECORD_CACHE_MAX_LENGTH = 20000, :40) fed by a partition queue of at most 32
// (LazyFileReader.cs:12-14), so a file of any size streams through fixed memory.  ppg_cursor is
// that surface over the GPU path: the file is cut into batches of whole chunks of at most
// batch_bytes of text; each batch is read (pread into pinned memory), copied to HBM, decoded
// (inflate + record scan, the DecompressAll kernels) and brought back as the chunks' raw bytes
// (offset_k ++ chunk_k, Parsing.cs's CombinedMemory) plus the record descriptors.
//
// What bounds it is PCIe: every byte of text crosses device -> host once (~385 B per record at
// 150 bp), the compressed input host -> device in the other direction.  So several batches are in
// flight, each on its own stream and worker thread, in stage order: while the caller walks batch
// k, batch k+1 crosses PCIe, k+2 decodes and k+3 is read, and the device -> host copies run back
// to back (r03: 122 M records/s, 86% of the PCIe bound).  Every slot's buffers -- pinned text /
// descriptor / compressed staging, device input, output, census, and the shard's own -- are sized
// once at open from the largest batch, so no worker reallocates (a hipFree waits for the whole
// device: 300-560 ms stalls per batch before r03's shard_reserve).  A batch's raw_k are packed on
// the device (ppg_pack_raw) and cross PCIe as one copy.  An index with side points
// (ppg_index_build_gpu_side) splits a batch's chunks into several waves when the batch is too
// small to fill the GPU by itself.
//
// A batch stays valid until the next ppg_cursor_next call (the reference's records are likewise
// invalid after the next MoveNext, BatchedFASTQ.cs:56 / SURVEY Q9).  Order is canonical (chunk 0's
// records, then chunk 1's, ...), not the reference's interleaving.
#include "ppg_host.h"
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

// launcher (ppg_parse.hip)
hipError_t ppg_launch_pack_raw(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs, const PpgInflateResult *ires,
                               const uint8_t *offs, const PpgOffsetRef *oref, const int64_t *raw_off, uint8_t *dst,
                               int n, int blocks);
hipError_t ppg_launch_copy16(hipStream_t s, const void *src, void *dst, uint64_t n16, int blocks);

namespace {

constexpr int kMaxSlots = 8;   // batches held: 5 by default (4 in flight + the caller's), PPG_CURSOR_SLOTS 2..8

struct Slot {
    ppg_shard sh;                       // device state of the batch (its own stream)
    DevBuf<uint8_t> dcomp;              // the batch's compressed bytes in HBM
    PinnedBuf pcomp;                    // ... staged in pinned host memory
    PinnedBuf text;                     // raw_k = offset_k ++ chunk_k, concatenated
    DevBuf<uint8_t> dtext;              // ... packed on the device first (one D2H per batch)
    DevBuf<int64_t> draw_off;
    PinnedBuf desc;                     // 4 x u32 per record
    std::vector<int64_t> raw_off, rec_off;
    int32_t b0 = 0, b1 = 0;             // chunks [b0, b1) relative to the cursor's first
    int64_t nrec = 0;
    int rc = PPG_OK;
    std::thread worker;
};

}  // namespace

// MemAvailable of /proc/meminfo in bytes (page cache included: it is reclaimable), or 0
static double host_mem_available() {
    FILE *f = fopen("/proc/meminfo", "r");
    if (!f) return 0;
    char line[256];
    double kb = 0;
    while (fgets(line, sizeof line, f))
        if (sscanf(line, "MemAvailable: %lf kB", &kb) == 1) break;
    fclose(f);
    return kb * 1024.0;
}

struct ppg_cursor {
    ppg_ctx *ctx = nullptr;
    const ppg_index *ix = nullptr;
    int fd = -1;
    int32_t first = 0, n = 0;
    int threads = 8;
    bool split = false;                 // batches smaller than ~6 generations of waves split at side points
    std::vector<std::pair<int32_t, int32_t>> batches;
    Slot slot[kMaxSlots];
    int nslots = 5;
    // how a batch's text and descriptors reach the host (PPG_CURSOR_PACK): 1 (default) packed on the
    // device, then one copy-engine copy at the PCIe rate; 0 one copy per chunk (~45 GB/s: 2,000+
    // small copies); 2 the pack kernel stores straight into the pinned buffers -- no copy engine,
    // but while those stores drain over PCIe the other batches' decode kernels do not complete
    // (decode 90 -> 250-440 ms with a pack in flight, any grid size, r03), so it loses
    int pack = 1;
    int pack_blocks = 256;              // pack = 2: workgroups of the pack kernels (PPG_CURSOR_PACK_BLOCKS)
    bool verbose = false;               // PPG_CURSOR_VERBOSE: per-batch stage times on stderr
    std::chrono::steady_clock::time_point t_open = std::chrono::steady_clock::now();
    size_t next = 0;                    // next batch to hand out
    int64_t record_base = 0;
    // stage order across batches: batch i reads only after batch i-1 has read, and starts its
    // device -> host transfer only after batch i-1's has completed.  Without it the batches in
    // flight start together and move in lockstep -- all reading, then all decoding, then all
    // copying -- and PCIe idles between the groups (r03: 3 batches started at once, ~90 M
    // records/s); in order, batch i+1 reads and decodes while batch i crosses PCIe.
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint8_t> stage;         // per batch: kRead | kHost once that stage is over (or failed)
    static constexpr uint8_t kRead = 1, kHost = 2;
    void stage_done(size_t i, uint8_t bit) {
        std::lock_guard<std::mutex> lk(mu);
        stage[i] |= bit;
        cv.notify_all();
    }
    void stage_wait(size_t i, uint8_t bit) {   // for batch i-1's stage
        if (i == 0) return;
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return (stage[i - 1] & bit) != 0; });
    }

    ~ppg_cursor() {
        for (auto &s : slot)
            if (s.worker.joinable()) s.worker.join();   // (slots past nslots never started)
        (void)hipSetDevice(ctx->device);
        for (auto &s : slot) {
            for (auto &e : s.sh.ev) if (e) (void)hipEventDestroy(e);
            if (s.sh.h_tot) (void)hipHostFree(s.sh.h_tot);
            if (s.sh.stream) (void)hipStreamDestroy(s.sh.stream);
            s.sh.h_tot = nullptr;
            for (auto &e : s.sh.ev) e = nullptr;
        }
        if (fd >= 0) close(fd);
    }

    int64_t comp_len(size_t i) const {
        const auto &P = ix->pts;
        return P[(size_t)(first + batches[i].second)].input - P[(size_t)(first + batches[i].first)].input + 1;
    }
    int64_t raw_len(size_t i) const {
        const auto &P = ix->pts;
        int64_t t = 0;
        for (int32_t k = first + batches[i].first; k < first + batches[i].second; k++)
            t += (P[(size_t)k + 1].output - P[(size_t)k].output) + (int64_t)P[(size_t)k].offset.size();
        return t;
    }

    // every slot's buffers, once, for the largest batch -- the shard's device buffers too
    // (shard_reserve): a reallocation in a worker frees first, and hipFree waits for the device
    int size_slots() {
        int64_t cmax = 1, rmax = 1, max_chunks = 1;
        for (size_t i = 0; i < batches.size(); i++) {
            max_chunks = std::max<int64_t>(max_chunks, batches[i].second - batches[i].first);
            cmax = std::max(cmax, comp_len(i));
            rmax = std::max(rmax, raw_len(i));
        }
        // every slot holds its largest batch pinned on the host (compressed bytes, raw text,
        // descriptors) and on the device (the same + the shard's output, census and records):
        // fewer slots (not below 2) when they would take more than half the available host memory
        // or 80% of the free device memory (at 4 GiB batches, 5 slots are ~28 GB pinned)
        const double host_slot = (double)cmax + (double)rmax * 1.125;
        const double dev_slot = (double)cmax + (double)rmax * (pack == 1 ? 2.4 : 1.4);
        size_t dfree = 0, dtotal = 0;
        const double havail = host_mem_available();
        if (hipMemGetInfo(&dfree, &dtotal) != hipSuccess) dfree = 0;
        while (nslots > 2 && ((havail > 0 && nslots * host_slot > 0.5 * havail) ||
                              (dfree > 0 && nslots * dev_slot > 0.8 * (double)dfree)))
            nslots--;
        for (int q = 0; q < nslots; q++) {
            Slot &s = slot[q];
            HIPCHK(s.pcomp.alloc((size_t)cmax));
            HIPCHK(s.dcomp.alloc((size_t)cmax + 64));
            HIPCHK(s.text.alloc((size_t)rmax));
            if (pack) HIPCHK(s.draw_off.alloc((size_t)max_chunks + 1));
            if (pack == 1) HIPCHK(s.dtext.alloc((size_t)rmax));
            // descriptors: 16 B per record, for records of >= 128 B on average (grown only beyond)
            HIPCHK(s.desc.alloc((size_t)(rmax / 8 + 4096)));
            if (int rc = shard_reserve(&s.sh, ix, first, batches, split)) return rc;
        }
        return PPG_OK;
    }

    // read, decode and bring back batch i into slot s (runs on the slot's worker thread)
    int produce(size_t i, Slot &s) {
        using Clk = std::chrono::steady_clock;
        const auto t0 = Clk::now();
        auto ms = [&] { return std::chrono::duration<double, std::milli>(Clk::now() - t0).count(); };
        double tr = 0, tp = 0, td = 0;
        struct Done {   // every exit, failures included, releases the next batch's waits
            ppg_cursor *c; size_t i;
            ~Done() { c->stage_done(i, kRead | kHost); }
        } done{this, i};
        if (hipSetDevice(ctx->device) != hipSuccess) return PPG_DEVICE_ERROR;
        const auto &P = ix->pts;
        const int32_t a = first + batches[i].first, b = first + batches[i].second;
        s.b0 = batches[i].first;
        s.b1 = batches[i].second;
        const int64_t lo = P[(size_t)a].input - 1, len = comp_len(i);
        stage_wait(i, kRead);
        const double tw = ms();
        if (!pread_parallel(fd, s.pcomp.p, lo, len, threads)) return PPG_IO_ERROR;
        stage_done(i, kRead);
        tr = ms();
        hipStream_t st = s.sh.stream;
        HIPCHK(hipMemsetAsync(s.dcomp.p + len, 0, 64, st));
        HIPCHK(hipMemcpyAsync(s.dcomp.p, s.pcomp.p, (size_t)len, hipMemcpyHostToDevice, st));
        if (int rc = shard_prepare(&s.sh, ix, a, b - a, s.dcomp.p, len, 0, st)) return rc;
        if (split)
            if (int rc = shard_split_from_index(&s.sh, ix, a, b - a)) return rc;
        shard_reset(&s.sh);
        tp = ms();
        float kms = 0;
        if (int rc = batch_launch(&s.sh, 0, s.sh.n)) return rc;
        if (int rc = batch_collect(&s.sh, 0, s.sh.n, kms)) return rc;
        if (int rc = shard_finish(&s.sh, kms)) return rc;
        td = ms();
        // raw_k = offset_k ++ chunk_k (Parsing.Parse's CombinedMemory), back to pinned host memory
        const int32_t m = b - a;
        s.raw_off.assign((size_t)m + 1, 0);
        for (int32_t k = 0; k < m; k++)
            s.raw_off[(size_t)k + 1] = s.raw_off[(size_t)k] + (int64_t)P[(size_t)a + k].offset.size() +
                                       (int64_t)s.sh.h_res[(size_t)k].produced;
        if ((size_t)s.raw_off[(size_t)m] > s.text.n) return PPG_BUF_ERROR;   // produced <= Output span: never
        s.nrec = s.sh.total_records;
        if ((size_t)(16 * s.nrec) > s.desc.n) HIPCHK(s.desc.alloc((size_t)(16 * s.nrec + (16 * s.nrec) / 4)));
        stage_wait(i, kHost);
        const double th = ms();
        if (pack == 2) {
            // raw_k = offset_k ++ chunk_k stored by the pack kernel straight into the pinned text
            // buffer, the descriptors likewise: the copy engines stay free for the host -> device
            // direction of the other batches (SDMA copies of the two directions serialised, r03:
            // tools/pcie_probe.hip)
            HIPCHK(hipMemcpyAsync(s.draw_off.p, s.raw_off.data(), 8 * ((size_t)m + 1), hipMemcpyHostToDevice, st));
            HIPCHK(ppg_launch_pack_raw(st, s.sh.out.p, s.sh.jobs.p, s.sh.res.p, s.sh.offs.p, s.sh.oref.p,
                                       s.draw_off.p, s.text.p, m, pack_blocks));
            HIPCHK(ppg_launch_copy16(st, s.sh.recs.p, s.desc.p, (uint64_t)s.nrec, pack_blocks));
        } else if (pack == 1) {
            // packed on the device, then the batch's text crosses PCIe as one copy
            HIPCHK(hipMemcpyAsync(s.draw_off.p, s.raw_off.data(), 8 * ((size_t)m + 1), hipMemcpyHostToDevice, st));
            HIPCHK(ppg_launch_pack_raw(st, s.sh.out.p, s.sh.jobs.p, s.sh.res.p, s.sh.offs.p, s.sh.oref.p,
                                       s.draw_off.p, s.dtext.p, m, 0));
            if (s.raw_off[(size_t)m])
                HIPCHK(hipMemcpyAsync(s.text.p, s.dtext.p, (size_t)s.raw_off[(size_t)m], hipMemcpyDeviceToHost, st));
        } else {
            // the chunks' bodies are contiguous on the device; each lands after its offset carry
            // (one copy per chunk measured faster than packing + one copy: 98 vs 85 M records/s, r03)
            for (int32_t k = 0; k < m; k++) {
                const auto &off = P[(size_t)a + k].offset;
                uint8_t *dst = s.text.p + s.raw_off[(size_t)k];
                if (!off.empty()) memcpy(dst, off.data(), off.size());
                const uint64_t got = s.sh.h_res[(size_t)k].produced;
                if (got) HIPCHK(hipMemcpyAsync(dst + off.size(), s.sh.out.p + s.sh.h_jobs[(size_t)k].out_off, got,
                                               hipMemcpyDeviceToHost, st));
            }
        }
        if (s.nrec && pack != 2)
            HIPCHK(hipMemcpyAsync(s.desc.p, s.sh.recs.p, 16 * (size_t)s.nrec, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        stage_done(i, kHost);
        if (verbose)
            fprintf(stderr, "[cursor] batch %zu: %d chunks, started at %.1f ms: read wait %.1f, read %.1f, H2D+prepare %.1f, "
                            "decode %.1f (kernels %.1f), host wait %.1f, to host %.1f, total %.1f ms\n", i, m,
                    std::chrono::duration<double, std::milli>(t0 - t_open).count(), tw, tr - tw, tp - tr, td - tp,
                    (double)kms, th - td, ms() - th, ms());
        s.rec_off.assign((size_t)m + 1, 0);
        for (int32_t k = 0; k < m; k++) s.rec_off[(size_t)k + 1] = s.sh.h_base[(size_t)k] + (int64_t)s.sh.h_info[(size_t)k].records;
        return PPG_OK;
    }

    void start(size_t i) {
        Slot &s = slot[i % (size_t)nslots];
        s.rc = PPG_OK;
        s.worker = std::thread([this, i, &s] { s.rc = produce(i, s); });
    }
};

extern "C" {

int ppg_cursor_open(ppg_ctx *ctx, const ppg_index *ix, const char *gz_path, int32_t first, int32_t n,
                    int64_t batch_bytes, int threads, ppg_cursor **out) {
    if (!ctx || !ix || !gz_path || !out || first < 0 || n < 0 || (size_t)first + (size_t)n + 1 > ix->pts.size())
        return PPG_ARG_ERROR;
    if (int v = ppg_index_validate(ix, first, n)) return v;
    if (batch_bytes <= 0) batch_bytes = (int64_t)1 << 30;   // callers wanting throughput ask for more (bench: 8 GiB)
    HIPCHK(hipSetDevice(ctx->device));
    auto c = std::make_unique<ppg_cursor>();
    c->ctx = ctx;
    c->ix = ix;
    c->first = first;
    c->n = n;
    c->threads = threads > 0 ? threads : 8;
    if (const char *e = getenv("PPG_CURSOR_SLOTS")) c->nslots = std::min(kMaxSlots, std::max(2, atoi(e)));
    if (const char *e = getenv("PPG_CURSOR_PACK")) c->pack = std::min(2, std::max(0, atoi(e)));
    if (const char *e = getenv("PPG_CURSOR_PACK_BLOCKS")) c->pack_blocks = std::max(4, atoi(e));
    c->verbose = getenv("PPG_CURSOR_VERBOSE") != nullptr;
    c->fd = open(gz_path, O_RDONLY);
    if (c->fd < 0) return PPG_IO_ERROR;
    // batches: whole chunks, at most batch_bytes of raw text each (at least one chunk)
    const auto &P = ix->pts;
    int32_t max_chunks = 0;
    for (int32_t a = 0; a < n;) {
        int32_t b = a + 1;
        int64_t raw = (P[(size_t)first + a + 1].output - P[(size_t)first + a].output) + (int64_t)P[(size_t)first + a].offset.size();
        while (b < n) {
            const int64_t r = (P[(size_t)first + b + 1].output - P[(size_t)first + b].output) +
                              (int64_t)P[(size_t)first + b].offset.size();
            if (raw + r > batch_bytes) break;
            raw += r;
            b++;
        }
        c->batches.push_back({a, b});
        max_chunks = std::max(max_chunks, b - a);
        a = b;
    }
    if (!ix->side_out.empty()) {   // the ~6 generations of waves the bench's auto split uses
        int cus = 0;
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
        c->split = (int64_t)max_chunks < 6 * 32 * (int64_t)cus;
    }
    for (int q = 0; q < c->nslots; q++) {
        c->slot[q].sh.ctx = ctx;
        HIPCHK(hipStreamCreateWithFlags(&c->slot[q].sh.stream, hipStreamNonBlocking));
    }
    if (int rc = c->size_slots()) return rc;
    c->stage.assign(c->batches.size(), 0);
    for (size_t i = 0; i < c->batches.size() && i < (size_t)c->nslots - 1; i++) c->start(i);
    *out = c.release();
    return PPG_OK;
}

int ppg_cursor_next(ppg_cursor *c, ppg_batch *b) {
    if (!c || !b) return PPG_ARG_ERROR;
    if (c->next >= c->batches.size()) return PPG_STREAM_END;
    const size_t S = (size_t)c->nslots;
    Slot &s = c->slot[c->next % S];
    if (s.worker.joinable()) s.worker.join();
    if (s.rc != PPG_OK) return s.rc;
    // the slot of the batch handed out last time is free again: the caller is done with it
    if (c->next + S - 1 < c->batches.size()) {
        Slot &f = c->slot[(c->next + S - 1) % S];
        if (f.worker.joinable()) f.worker.join();
        c->start(c->next + S - 1);
    }
    b->first_chunk = c->first + s.b0;
    b->nchunks = s.b1 - s.b0;
    b->record_base = c->record_base;
    b->nrecords = s.nrec;
    b->text = s.text.p;
    b->raw_off = s.raw_off.data();
    b->desc = (const uint32_t *)s.desc.p;
    b->rec_off = s.rec_off.data();
    c->record_base += s.nrec;
    c->next++;
    return PPG_OK;
}

int32_t ppg_cursor_batches(const ppg_cursor *c) { return c ? (int32_t)c->batches.size() : -1; }

void ppg_cursor_close(ppg_cursor *c) { delete c; }

}  // extern "C"

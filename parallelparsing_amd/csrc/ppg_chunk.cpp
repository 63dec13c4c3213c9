// ppg_chunk.cpp — README "Decompress": one checkpoint at a time, thread safe
// (/root/reference/README.md:38-50 "must be thread safe"; Core.ExtractDeflateIndex,
// Decompressor/Core.cs:133-192, + Parsing.Parse as BatchedFASTQ.cs:63-74 runs them per task).
//
// The reference calls this once per chunk from a ThreadPool task per chunk (BatchedFASTQ.cs:62-77),
// each with its own ZStream.  On the GPU one chunk alone is one wave of the 8,192 the chip holds,
// so concurrent calls are *combined*: a call queues its request, and whichever waiting caller finds
// one of the ctx's two launch slots free takes every queued request into one launch (flat
// combining -- no service thread).  While a launch runs, new calls queue up for the other slot, so
// T callers keep up to T chunks in flight in at most two launches.
//
// A slot owns everything a launch touches -- its stream, a one-batch ppg_shard, the gathered
// compressed slices (pinned + device), the pinned copy of the outputs and descriptors -- and its
// buffers only grow (geometrically), so a warm ctx makes no hipMalloc/hipFree per call: hipFree
// waits for the whole device.  Each caller copies its own chunk out of the slot's pinned results
// in parallel with the others; the slot is reused only after every such copy is done.
//
// Chunks whose index carries side points (ppg_index_build_gpu_side) are decoded as one wave per
// piece between their inner block starts (ppg_shard_set_split), exactly as DecompressAll does.
#include "ppg_host.h"
#include <condition_variable>
#include <deque>
#include <mutex>

namespace {

constexpr int kChunkSlots = 2;
constexpr size_t kSliceAlign = 64;   // each gathered slice starts on its own 64-B line

struct ChunkReq {
    const ppg_index *ix;
    int32_t k;
    const uint8_t *slice;
    int64_t slice_len;
    // results, set by the launching caller
    bool done = false;
    int rc = PPG_OK;
    int slot = -1;
    const uint8_t *src = nullptr;       // chunk bytes in the slot's pinned results
    int64_t got = 0;
    const uint32_t *src_recs = nullptr;
    int64_t nrec = 0;
};

// grow a buffer to `need` elements, by at least half again its size (no reallocation per call)
template <class B>
hipError_t grow_buf(B &b, size_t need) {
    if (b.p && b.n >= need) return hipSuccess;
    return b.alloc(std::max(need, b.n + b.n / 2));
}

struct ChunkSlot {
    hipStream_t s = nullptr;
    ppg_shard *sh = nullptr;
    PinnedBuf in;                       // the launch's slices, gathered
    DevBuf<uint8_t> comp;
    PinnedBuf res;                      // outputs, then descriptors
    bool busy = false;
    int readers = 0;                    // callers still copying out of `res`
};

}  // namespace

struct ChunkService {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<ChunkReq *> pending;
    ChunkSlot slot[kChunkSlots];
    int64_t calls = 0, launches = 0, max_batch = 0;
};

ChunkService *chunk_service_new() { return new ChunkService; }

void chunk_service_free(ChunkService *svc) {
    if (!svc) return;
    for (auto &sl : svc->slot) {
        if (sl.sh) ppg_shard_free(sl.sh);
        if (sl.s) (void)hipStreamDestroy(sl.s);
    }
    delete svc;
}

namespace {

// side points of chunk k of ix (strictly inside it), in the launch's virtual coordinates: output =
// the chunk's offset in the launch output + its own offset, bit = the chunk's job bit + the same
// distance in the file
void side_points_of(const ppg_index *ix, int32_t k, uint64_t job_bit, int64_t out_base, std::vector<int64_t> &bit,
                    std::vector<int64_t> &out, ByteVec &win) {
    const auto &O = ix->side_out;
    if (O.empty()) return;
    const PpgPoint &from = ix->pts[(size_t)k], &to = ix->pts[(size_t)k + 1];
    const int64_t from_bit = 8 * from.input - from.bits;
    const size_t a = (size_t)(std::upper_bound(O.begin(), O.end(), from.output) - O.begin());
    const size_t b = (size_t)(std::lower_bound(O.begin(), O.end(), to.output) - O.begin());
    for (size_t q = a; q < b; q++) {
        bit.push_back((int64_t)job_bit + (ix->side_bit[q] - from_bit));
        out.push_back(out_base + (O[q] - from.output));
        win.insert(win.end(), ix->side_win.data() + q * kWin, ix->side_win.data() + (q + 1) * kWin);
    }
}

// One launch of the requests `batch` on slot `sl` (the caller holds the slot, not the lock).  Sets
// every request's rc and, for a decoded chunk, where its bytes and descriptors sit in sl.res.
int run_launch(ppg_ctx *ctx, ChunkSlot &sl, std::vector<ChunkReq *> &batch) {
    HIPCHK(hipSetDevice(ctx->device));
    if (!sl.s) HIPCHK(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
    if (!sl.sh) {
        sl.sh = new ppg_shard;
        sl.sh->ctx = ctx;
        sl.sh->stream = sl.s;
    }
    // requests the kernels can take, laid out slice after slice
    std::vector<ChunkReq *> go;
    std::vector<ChunkSpec> spec;
    std::vector<int64_t> at;
    size_t comp_len = 0;
    for (ChunkReq *r : batch) {
        const auto &P = r->ix->pts;
        int rc = ppg_index_validate(r->ix, r->k, 1);
        if (rc == PPG_OK && r->slice_len != P[(size_t)r->k + 1].input - P[(size_t)r->k].input + 1) rc = PPG_ARG_ERROR;
        if (rc == PPG_OK && r->ix->windows.size() < ((size_t)r->k + 1) * kWin) rc = PPG_ARG_ERROR;
        if (rc != PPG_OK) {
            r->rc = rc;
            continue;
        }
        go.push_back(r);
        at.push_back((int64_t)comp_len);
        spec.push_back(ChunkSpec{&P[(size_t)r->k], &P[(size_t)r->k + 1], r->ix->win((size_t)r->k), (int64_t)comp_len,
                                 (size_t)r->k + 2 == P.size()});
        comp_len += ((size_t)r->slice_len + kSliceAlign - 1) / kSliceAlign * kSliceAlign;
    }
    if (go.empty()) return PPG_OK;
    {   // the shard's buffers with headroom, so launches of growing size do not reallocate each time
        size_t n = go.size(), offb = 0, tot = 0, nsub = 0;
        for (ChunkReq *r : go) {
            const PpgPoint &from = r->ix->pts[(size_t)r->k], &to = r->ix->pts[(size_t)r->k + 1];
            offb += from.offset.size();
            tot += (size_t)std::max<int64_t>(to.output - from.output, 0);
            const auto &O = r->ix->side_out;
            nsub += (size_t)std::max<std::ptrdiff_t>(0, std::lower_bound(O.begin(), O.end(), to.output) -
                                                            std::upper_bound(O.begin(), O.end(), from.output));
        }
        ppg_shard *sh = sl.sh;
        HIPCHK(grow_buf(sh->jobs, n));
        HIPCHK(grow_buf(sh->dicts, (n + nsub) * kWin));
        HIPCHK(grow_buf(sh->offs, offb + 16));
        HIPCHK(grow_buf(sh->oref, n));
        HIPCHK(grow_buf(sh->res, n));
        HIPCHK(grow_buf(sh->info, n));
        HIPCHK(grow_buf(sh->base, n));
        HIPCHK(grow_buf(sh->total, 1));
        HIPCHK(grow_buf(sh->out, tot + 64));
        HIPCHK(grow_buf(sh->recs, 4 * (tot / 256 + 1024)));
        HIPCHK(grow_buf(sh->nls, 2 * (tot / kNlBytesPerEntry + 64 * (n + nsub)) + 64));
        if (nsub) {
            HIPCHK(grow_buf(sh->sjobs, n + nsub));
            HIPCHK(grow_buf(sh->sres, n + nsub));
            HIPCHK(grow_buf(sh->sidx, n + 1));
        }
    }
    HIPCHK(grow_buf(sl.in, comp_len + 256));
    HIPCHK(grow_buf(sl.comp, comp_len + 256));
    memset(sl.in.p, 0, comp_len + 256);
    for (size_t i = 0; i < go.size(); i++) memcpy(sl.in.p + at[i], go[i]->slice, (size_t)go[i]->slice_len);
    HIPCHK(hipMemcpyAsync(sl.comp.p, sl.in.p, comp_len + 256, hipMemcpyHostToDevice, sl.s));
    ppg_shard *sh = sl.sh;
    int rc = shard_prepare_specs(sh, spec.data(), (int32_t)go.size(), sl.comp.p, (int64_t)comp_len, 0, sl.s, nullptr);
    if (rc != PPG_OK) return rc;
    {   // side points of the chunks that have them (the index's, shifted into this launch)
        std::vector<int64_t> sbit, sout;
        ByteVec swin;
        for (size_t i = 0; i < go.size(); i++)
            side_points_of(go[i]->ix, go[i]->k, sh->h_jobs[i].bit_start, sh->h_pout[i], sbit, sout, swin);
        if (!sbit.empty()) {
            rc = ppg_shard_set_split(sh, (int32_t)sbit.size(), sbit.data(), sout.data(), swin.data());
            if (rc != PPG_OK) return rc;
        }
    }
    shard_reset(sh);
    float total_ms = 0;
    if ((rc = batch_launch(sh, 0, sh->n)) != PPG_OK) return rc;
    if ((rc = batch_collect(sh, 0, sh->n, total_ms)) != PPG_OK) return rc;
    // shard_finish returns the first chunk's zlib status (each request gets its own below) or a
    // device failure, which fails every request of the launch
    if ((rc = shard_finish(sh, total_ms)) <= PPG_INDEX_OUT_OF_RANGE) return rc;
    // results: the whole output, then every descriptor, into the slot's pinned buffer
    const size_t out_bytes = (size_t)sh->h_pout[(size_t)sh->n];
    const size_t rec_bytes = 16 * (size_t)sh->total_records;
    const size_t rec_at = (out_bytes + 15) / 16 * 16;
    HIPCHK(grow_buf(sl.res, rec_at + rec_bytes + 16));
    if (out_bytes) HIPCHK(hipMemcpyAsync(sl.res.p, sh->out.p, out_bytes, hipMemcpyDeviceToHost, sl.s));
    if (rec_bytes) HIPCHK(hipMemcpyAsync(sl.res.p + rec_at, sh->recs.p, rec_bytes, hipMemcpyDeviceToHost, sl.s));
    HIPCHK(hipStreamSynchronize(sl.s));
    for (size_t i = 0; i < go.size(); i++) {
        ChunkReq *r = go[i];
        const PpgInflateResult &res = sh->h_res[i];
        r->rc = res.status;
        r->got = (int64_t)res.produced;
        r->src = sl.res.p + sh->h_jobs[i].out_off;
        r->nrec = (int64_t)sh->h_info[i].records;
        r->src_recs = (const uint32_t *)(sl.res.p + rec_at) + 4 * sh->h_base[i];
    }
    return PPG_OK;
}

}  // namespace

extern "C" {

// README "Decompress" (see the top of this file).  Safe to call from any number of host threads
// on one ctx at once.
int ppg_decompress_chunk(ppg_ctx *ctx, const ppg_index *ix, int32_t k, const uint8_t *slice, int64_t slice_len,
                         uint8_t *out, int64_t out_cap, int64_t *produced, uint32_t *recs, int64_t rec_cap,
                         int64_t *nrec) {
    if (!ctx || !ix || !slice || k < 0 || (size_t)k + 1 >= ix->pts.size() || !ctx->chunks) return PPG_ARG_ERROR;
    ChunkService *svc = ctx->chunks;
    ChunkReq req{ix, k, slice, slice_len};
    std::unique_lock<std::mutex> lk(svc->mu);
    svc->calls++;
    svc->pending.push_back(&req);
    while (!req.done) {
        int free_slot = -1;
        for (int i = 0; i < kChunkSlots && free_slot < 0; i++)
            if (!svc->slot[i].busy && svc->slot[i].readers == 0) free_slot = i;
        if (free_slot < 0 || svc->pending.empty()) {
            svc->cv.wait(lk);
            continue;
        }
        // lead a launch of every queued request (this one among them, unless another caller took it)
        std::vector<ChunkReq *> batch(svc->pending.begin(), svc->pending.end());
        svc->pending.clear();
        ChunkSlot &sl = svc->slot[free_slot];
        sl.busy = true;
        svc->launches++;
        svc->max_batch = std::max<int64_t>(svc->max_batch, (int64_t)batch.size());
        lk.unlock();
        const int rc = run_launch(ctx, sl, batch);
        lk.lock();
        for (ChunkReq *r : batch) {
            if (rc != PPG_OK) r->rc = rc;
            if (r->rc == PPG_OK) {
                r->slot = free_slot;
                sl.readers++;
            }
            r->done = true;
        }
        sl.busy = false;
        svc->cv.notify_all();
    }
    lk.unlock();
    // copy this chunk out of the slot's pinned results (callers copy in parallel)
    int rc = req.rc;
    if (rc == PPG_OK) {
        int64_t len = req.got;
        if (out) {
            if (req.got > out_cap) {
                rc = PPG_BUF_ERROR;
                len = 0;
            } else if (req.got) {
                memcpy(out, req.src, (size_t)req.got);
            }
        }
        if (produced) *produced = len;
        if (rc == PPG_OK) {
            if (nrec) *nrec = req.nrec;
            if (recs) {
                if (req.nrec > rec_cap) rc = PPG_BUF_ERROR;
                else if (req.nrec) memcpy(recs, req.src_recs, 16 * (size_t)req.nrec);
            }
        }
        lk.lock();
        if (--svc->slot[req.slot].readers == 0) svc->cv.notify_all();
    }
    return rc;
}

int ppg_decompress_chunk_stats(ppg_ctx *ctx, int64_t *calls, int64_t *launches, int64_t *max_batch) {
    if (!ctx || !ctx->chunks) return PPG_ARG_ERROR;
    std::lock_guard<std::mutex> lk(ctx->chunks->mu);
    if (calls) *calls = ctx->chunks->calls;
    if (launches) *launches = ctx->chunks->launches;
    if (max_batch) *max_batch = ctx->chunks->max_batch;
    return PPG_OK;
}

}  // extern "C"

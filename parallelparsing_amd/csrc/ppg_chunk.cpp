// ppg_chunk.cpp — README "Decompress": one checkpoint at a time, thread safe
// (/root/reference/README.md:38-50 "must be thread safe"; Core.ExtractDeflateIndex,
// Decompressor/Core.cs:133-192, + Parsing.Parse as BatchedFASTQ.cs:63-74 runs them per task).
//
// The reference calls this once per chunk from a ThreadPool task per chunk (BatchedFASTQ.cs:62-77),
// each with its own ZStream.  On the GPU one chunk alone is one wave of the 8,192 the chip holds,
// so concurrent calls are *combined*: a call queues its request, and whichever waiting caller finds
// one of the ctx's four launch slots free takes the queued requests (up to 256) into one launch
// (flat combining).  A second launch starts beside a running one only once 16 requests queue, so
// the queue that builds during a launch goes into the next one.  Asynchronous requests
// (ppg_decompress_chunk_submit) are launched the same way by a launcher thread of the ctx, and
// their results copied out by a copier thread while the next launch runs.
//
// A slot owns everything a launch touches -- its stream, a one-batch ppg_shard, the gathered
// compressed slices (pinned + device), the pinned copy of the outputs and descriptors, the block
// search's scratch -- and its buffers only grow (geometrically), so a warm ctx makes no
// hipMalloc/hipFree per call: hipFree waits for the whole device.  Each synchronous caller copies
// its own chunk out of the slot's pinned results in parallel with the others; the slot is reused
// only after every such copy is done.
//
// Chunks whose index carries side points (ppg_index_build_gpu_side) are decoded as one wave per
// piece between their inner block starts (ppg_shard_set_split), exactly as DecompressAll does; the
// others get theirs found on the GPU (find_side_points, find_mat below).
#include "ppg_host.h"
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <sys/mman.h>

hipError_t ppg_launch_block_find(hipStream_t s, const uint32_t *comp, uint64_t nwords, const uint64_t *lo,
                                 const uint64_t *hi, uint64_t *cand, int n, int sub);
hipError_t ppg_launch_inflate_ix(hipStream_t s, const uint32_t *comp, uint64_t nwords, const PpgInflateJob *jobs,
                                 const uint8_t *dicts, uint8_t *out, PpgInflateResult *res, PpgBlockEnd *blk,
                                 int njobs);
hipError_t ppg_launch_inflate_ixf(hipStream_t s, const uint32_t *comp, uint64_t nwords, const PpgInflateJob *jobs,
                                  const uint8_t *dicts, uint8_t *out, PpgInflateResult *res, PpgBlockEnd *blk,
                                  int njobs);
hipError_t ppg_launch_gather(hipStream_t s, const uint8_t *out, const uint8_t *dicts, const PpgGather *g, uint8_t *dst,
                             const uint8_t *ref, uint32_t *diff, int n);
hipError_t ppg_launch_resolve_chains(hipStream_t s, const uint8_t *ta, const uint32_t *slots, const uint4 *chains,
                                     int nchains, const uint8_t *windows, uint8_t *W);
hipError_t ppg_launch_pick_windows(hipStream_t s, const uint8_t *src, const uint32_t *idx, int n, uint8_t *dst);

namespace {

constexpr int kChunkSlots = 4;             // launches in flight / results being copied out
constexpr uint64_t kPieceRing = 65536;     // CreateIndex pass 1's symbolic output ring per piece (IX_RING_BYTES)
// launches of up to this many chunks split them at their inner block starts found on the GPU: ~16
// waves per chunk, so 4,096 chunks already hold ~8 generations of the GPU's 8,192 wave slots
constexpr int kFindMaxChunks = 4096;
constexpr size_t kSliceAlign = 64;   // each gathered slice starts on its own 64-B line
// chunks per launch: the materialise path's limit (find_mat, kMatMaxChunks below), whose launch of
// 256 warm chunks takes 41 ms against 63 ms for 258 on the two-decode path (r05g)
constexpr size_t kMaxBatch = 256;
// a second launch starts while one is decoding only with this many requests queued: otherwise the
// queue grows during the running launch and the next one takes all of it (r04: with two slots taken
// as soon as free, 64 callers were served ~12 at a time)
constexpr size_t kMinSecond = 16;
// launcher threads of asynchronous requests.  r05 (tools/chunk_latency.py, async depth 1024, three
// runs): one 19 / 31 / 39 M records/s, two 16 / 18 / 30 -- the second overlaps a launch's PCIe
// copies with the other's kernels, but the two launches' host copies (slices gathered, results
// copied out into fresh pages) then contend, and more slots are grown
constexpr int kLaunchers = 1;

struct ChunkReq {
    const ppg_index *ix;
    int32_t k;
    const uint8_t *slice;
    int64_t slice_len;
    // asynchronous requests (ppg_decompress_chunk_submit): where wait() copies the results
    bool async = false;
    uint8_t *out = nullptr;
    int64_t out_cap = 0;
    uint32_t *recs = nullptr;
    int64_t rec_cap = 0;
    // results, set by the launching caller
    bool done = false;
    int rc = PPG_OK;
    int slot = -1;
    const uint8_t *src = nullptr;       // chunk bytes in the slot's pinned results
    int64_t got = 0;
    const uint32_t *src_recs = nullptr;
    int64_t nrec = 0;
    // an async request's results already copied into out/recs by the launcher (fin_*: what wait() returns)
    bool copied = false;
    int fin_rc = PPG_OK;
    int64_t fin_len = 0;
    bool fin_nrec = false;
};

// grow a buffer to `need` elements, by at least half again its size (no reallocation per call)
template <class B>
hipError_t grow_buf(B &b, size_t need) {
    if (b.p && b.n >= need) return hipSuccess;
    return b.alloc(std::max(need, b.n + b.n / 2));
}

// memcpy of many (dst, src, len) spans: on the calling thread when small, else spread over up to
// 8 threads in 1 MiB pieces -- a launch gathers up to 256 slices into the pinned staging buffer and
// the async path copies up to a GiB of results into fresh caller pages (page faults included), which
// one thread does at a few GB/s
struct Span {
    uint8_t *dst;
    const uint8_t *src;
    size_t len;
};

void parallel_copy(const std::vector<Span> &v, bool caller_dst = false) {
    constexpr size_t kPiece = 1 << 20;
    size_t tot = 0;
    for (const Span &x : v) tot += x.len;
    if (tot < 8 * kPiece) {
        for (const Span &x : v)
            if (x.len) memcpy(x.dst, x.src, x.len);
        return;
    }
    // caller_dst: the caller's (often fresh) pages -- 2 MiB pages where a span covers them (advice
    // only, never on the slots' pinned buffers; r05, tools/chunk_latency.py: a 256-chunk launch's
    // 1 GB of results copied out in 30-36 ms instead of 62-70, async depth 256 30-33 M records/s
    // instead of 19-22)
    for (const Span &x : v) {
        if (!caller_dst) break;
        const uintptr_t a = ((uintptr_t)x.dst + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
        const uintptr_t b = ((uintptr_t)x.dst + x.len) & ~(uintptr_t)((2u << 20) - 1);
        if (b > a) (void)madvise((void *)a, b - a, MADV_HUGEPAGE);
    }
    std::vector<Span> pieces;
    for (const Span &x : v)
        for (size_t o = 0; o < x.len; o += kPiece) pieces.push_back(Span{x.dst + o, x.src + o, std::min(kPiece, x.len - o)});
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t i; (i = next.fetch_add(1)) < pieces.size();) memcpy(pieces[i].dst, pieces[i].src, pieces[i].len);
    };
    std::vector<std::thread> th;
    const size_t nt = std::min<size_t>(8, tot / (4 * kPiece));
    try {
        for (size_t t = 1; t < nt; t++) th.emplace_back(work);
    } catch (...) {   // no threads: the calling thread copies everything
    }
    work();
    for (auto &t : th) t.join();
}

// What a decoded request hands its caller: the status (PPG_BUF_ERROR when a buffer is too small),
// the byte count, whether the record count is reported, and the copies out of the slot's results.
int result_spans(const ChunkReq &req, uint8_t *out, int64_t out_cap, uint32_t *recs, int64_t rec_cap, int64_t &len,
                 bool &with_nrec, std::vector<Span> &cp) {
    len = req.got;
    with_nrec = false;
    if (out) {
        if (req.got > out_cap) {
            len = 0;
            return PPG_BUF_ERROR;
        }
        if (req.got) cp.push_back(Span{out, req.src, (size_t)req.got});
    }
    with_nrec = true;
    if (recs) {
        if (req.nrec > rec_cap) return PPG_BUF_ERROR;
        if (req.nrec) cp.push_back(Span{(uint8_t *)recs, (const uint8_t *)req.src_recs, 16 * (size_t)req.nrec});
    }
    return PPG_OK;
}

// grow a big scratch buffer of the block search; out of device memory (e.g. beside a resident
// DecompressAll shard) is not a failure of the requests: the caller decodes them whole instead
#define GROW_OR_SKIP(b, n)                                                                      \
    do {                                                                                        \
        const hipError_t grow_e = grow_buf(b, n);                                               \
        if (grow_e == hipErrorOutOfMemory) {                                                    \
            (void)hipGetLastError();                                                            \
            fprintf(stderr, "ppgpu: block search scratch %s of %zu elements: out of device memory, " \
                    "the launch's chunks decoded whole\n", #b, (size_t)(n));                   \
            return PPG_MEM_ERROR;                                                               \
        }                                                                                       \
        if (grow_e != hipSuccess) {                                                             \
            fprintf(stderr, "ppgpu: grow %s failed: %s\n", #b, hipGetErrorString(grow_e));     \
            return PPG_DEVICE_ERROR;                                                            \
        }                                                                                       \
    } while (0)

// waves per candidate range of the block search: enough for ~16,384 waves in all, two generations of
// the GPU's wave slots (a lone chunk's 48 ranges are searched by 32 waves each; r05: at 4,096 waves a
// launch of 256 chunks searched its 3,840 ranges with one wave each, 7.0 ms)
int find_sub(int ranges) { return std::max(1, std::min(32, 16384 / std::max(1, ranges))); }

// device scratch of find_side_points (grow only)
struct FindScratch {
    DevBuf<uint16_t> sym;                  // materialise path: every piece's pass-1 symbols, whole
    DevBuf<PpgMatInfo> mi;                 // ... and each materialised piece's info
    DevBuf<uint64_t> lo, hi, cand;
    DevBuf<PpgInflateJob> jobs;
    DevBuf<PpgInflateResult> res;
    DevBuf<PpgBlockEnd> blk;
    DevBuf<uint8_t> ring, ta, ident, W;
    DevBuf<PpgGather> gat;
    DevBuf<uint32_t> slots, pick;
    DevBuf<uint4> chains;
    DevBuf<uint8_t> packed;
};

struct ChunkSlot {
    hipStream_t s = nullptr;
    ppg_shard *sh = nullptr;
    PinnedBuf in;                       // the launch's slices, gathered
    DevBuf<uint8_t> comp;
    PinnedBuf res;                      // outputs, then descriptors
    FindScratch fs;
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
    int in_flight = 0;                                         // launches decoding now
    std::atomic<int64_t> found_chunks{0}, found_points{0};   // find_side_points' splits
    // the launcher of asynchronous requests (started by the first ppg_decompress_chunk_submit)
    ppg_ctx *ctx = nullptr;
    std::thread worker[kLaunchers];
    bool stop = false;
    std::chrono::steady_clock::time_point last_submit{};
    // the copier of asynchronous results: a launch's async requests are copied out here (holding a
    // reader on their slot) while the launcher leads the next launch on another slot
    struct CopyTask {
        int slot;
        std::vector<ChunkReq *> reqs;
    };
    std::deque<CopyTask> copies;
    std::thread copier;
};

ChunkService *chunk_service_new() { return new ChunkService; }

void chunk_service_free(ChunkService *svc) {
    if (!svc) return;
    {
        std::lock_guard<std::mutex> lk(svc->mu);
        svc->stop = true;
    }
    svc->cv.notify_all();
    for (auto &w : svc->worker)
        if (w.joinable()) w.join();
    if (svc->copier.joinable()) svc->copier.join();   // (it drains the queued copies first)
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

// The index's side points of chunk k lie strictly inside it in both output and compressed bits
// (side_points_of selects them by output).  Checked per request before the launch is built, so a bad
// side point fails only its own request, never the others sharing the launch (one bad
// point made ppg_shard_set_split fail the whole launch).
bool side_points_inside(const ppg_index *ix, int32_t k) {
    const auto &O = ix->side_out;
    if (O.empty()) return true;
    const PpgPoint &from = ix->pts[(size_t)k], &to = ix->pts[(size_t)k + 1];
    const int64_t from_bit = 8 * from.input - from.bits, to_bit = 8 * to.input - to.bits;
    const size_t a = (size_t)(std::upper_bound(O.begin(), O.end(), from.output) - O.begin());
    const size_t b = (size_t)(std::lower_bound(O.begin(), O.end(), to.output) - O.begin());
    int64_t prev = from_bit;
    for (size_t q = a; q < b; q++) {
        if (ix->side_bit[q] <= prev || ix->side_bit[q] >= to_bit) return false;
        prev = ix->side_bit[q];
    }
    return true;
}

// PPG_CHUNK_VERBOSE=1: a launch's phases (ms) on stderr -- where a lone chunk's latency goes
struct PhaseClock {
    bool on;
    std::chrono::steady_clock::time_point t0, t;
    char buf[512];
    int n = 0;
    PhaseClock() : on(getenv("PPG_CHUNK_VERBOSE") != nullptr) { t0 = t = std::chrono::steady_clock::now(); buf[0] = 0; }
    void mark(const char *what, hipStream_t s = nullptr) {
        if (!on) return;
        if (s) (void)hipStreamSynchronize(s);
        const auto now = std::chrono::steady_clock::now();
        n += snprintf(buf + n, sizeof buf - (size_t)n, " %s %.3f", what,
                      std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
        if (n >= (int)sizeof buf) n = (int)sizeof buf - 1;
    }
    // (at: the launch's start, ms on the steady clock -- overlapping launches of several slots line up)
    void dump(size_t reqs, int slot) {
        if (on)
            fprintf(stderr, "PPG_CHUNK launch of %zu: total %.3f ms: slot %d at %.3f:%s\n", reqs,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), slot,
                    std::chrono::duration<double, std::milli>(t0.time_since_epoch()).count(), buf);
    }
};

// Side points for chunks whose index has none (a .gzi carries only the Points): the inner deflate
// block starts of each chunk found on the GPU the way the GPU CreateIndex finds them
// (ppg_index_gpu.cpp) -- candidate dynamic-block headers every ~1/16 of the chunk's compressed bytes
// (ppg_block_find_kernel), each piece but the last decoded with symbolic output until a block ends
// at or past the next candidate (the inflate kernel's IX mode, the same kernels as CreateIndex pass
// 1), the chain of block ends walked from the chunk's own Point (a block end that is not the next
// candidate's start ends the chain there: that end is still a real block start), and the 32 KiB
// history at every verified block start resolved from the pieces' symbolic tails starting from the
// Point's window (ppg_resolve_*).  A lone chunk then decodes as ~16 waves instead of one: the
// speculative pass costs about one piece's decode, the split decode another.  Coordinates: bits in
// the launch's gathered comp buffer, outputs in the launch's output (the shard's virtual ones).
struct FindChunk {
    uint64_t bit0, bit1;                // compressed bits of the chunk: [from's start bit, slice end)
    uint64_t bit_end;                   // to's block start (8 to.Input - to.Bits), or bit1 for the last chunk
    int64_t out0;                       // the chunk's first output byte (launch coordinates)
    int64_t len;                        // the chunk's output bytes
    uint32_t win;                       // the Point's 32 KiB: window `win` of the shard's device dicts
};

int find_side_points(ChunkSlot &sl, const uint32_t *comp, uint64_t nwords, const uint8_t *dwin,
                     const std::vector<FindChunk> &ch,
                     std::vector<int64_t> &sbit, std::vector<int64_t> &sout, ByteVec &swin, int64_t &nsplit,
                     PhaseClock &clk) {
    hipStream_t s = sl.s;
    FindScratch &F = sl.fs;
    // candidates: the chunk cut into up to 16 pieces of >= 48 KiB of compressed bytes
    std::vector<uint64_t> lo, hi;
    std::vector<size_t> cfirst(ch.size() + 1, 0);
    for (size_t c = 0; c < ch.size(); c++) {
        const uint64_t span = ch[c].bit1 - ch[c].bit0;
        const uint64_t pb = std::max<uint64_t>(8ull * 48 * 1024, span / 16);
        for (uint64_t a = ch[c].bit0 + pb; a + 8ull * 1024 < ch[c].bit1; a += pb) {
            lo.push_back(a);
            hi.push_back(std::min(a + pb, ch[c].bit1));
        }
        cfirst[c + 1] = lo.size();
    }
    if (lo.empty()) return PPG_OK;
    const size_t nc = lo.size();
    HIPCHK(grow_buf(F.lo, nc));
    HIPCHK(grow_buf(F.hi, nc));
    HIPCHK(grow_buf(F.cand, nc));
    HIPCHK(hipMemcpyAsync(F.lo.p, lo.data(), 8 * nc, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(F.hi.p, hi.data(), 8 * nc, hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_block_find(s, comp, nwords, F.lo.p, F.hi.p, F.cand.p, (int)nc, find_sub((int)nc)));
    std::vector<uint64_t> cand(nc);
    HIPCHK(hipMemcpyAsync(cand.data(), F.cand.p, 8 * nc, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    clk.mark("f.cand");
    // pieces: chunk c's Point, then its candidates; every piece but the last decoded to the next
    struct Piece { size_t chunk; uint64_t start, stop; };
    std::vector<Piece> pc;
    std::vector<size_t> pfirst(ch.size() + 1, 0);
    for (size_t c = 0; c < ch.size(); c++) {
        std::vector<uint64_t> st{ch[c].bit0};
        for (size_t k = cfirst[c]; k < cfirst[c + 1]; k++)
            if (cand[k] != ~0ull && cand[k] > st.back()) st.push_back(cand[k]);
        for (size_t j = 0; j + 1 < st.size(); j++) pc.push_back({c, st[j], st[j + 1]});
        pfirst[c + 1] = pc.size();
    }
    const size_t np = pc.size();
    if (!np) return PPG_OK;
    std::vector<PpgInflateJob> jobs(np);
    uint64_t nblk = 0;
    for (size_t q = 0; q < np; q++) {
        PpgInflateJob &J = jobs[q];
        J = PpgInflateJob{};
        J.bit_start = pc[q].start;
        J.bit_limit = ch[pc[q].chunk].bit1;
        J.out_off = (uint64_t)q * kPieceRing;
        J.expect_end = ~0ull;
        J.stop_bit = pc[q].stop;
        J.blk_off = (uint32_t)nblk;
        J.blk_cap = (uint32_t)((pc[q].stop - pc[q].start) / 8 / 2048 + 64);
        nblk += J.blk_cap;
    }
    HIPCHK(grow_buf(F.jobs, np));
    HIPCHK(grow_buf(F.res, np));
    HIPCHK(grow_buf(F.blk, (size_t)nblk));
    HIPCHK(grow_buf(F.ring, np * 2 * kPieceRing));
    HIPCHK(grow_buf(F.ta, np * 2 * kWin));
    if (!F.ident.p) {   // u16 0..32767: position p < 0 of a piece is history symbol 32768 + p
        std::vector<uint16_t> id(kWin);
        for (int i = 0; i < kWin; i++) id[(size_t)i] = (uint16_t)i;
        HIPCHK(F.ident.alloc(2 * kWin));
        HIPCHK(hipMemcpyAsync(F.ident.p, id.data(), 2 * kWin, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(F.jobs.p, jobs.data(), sizeof(PpgInflateJob) * np, hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_inflate_ix(s, comp, nwords, F.jobs.p, F.ident.p, F.ring.p, F.res.p, F.blk.p, (int)np));
    std::vector<PpgInflateResult> res(np);
    std::vector<PpgBlockEnd> blk((size_t)nblk);
    HIPCHK(hipMemcpyAsync(res.data(), F.res.p, sizeof(PpgInflateResult) * np, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(blk.data(), F.blk.p, sizeof(PpgBlockEnd) * nblk, hipMemcpyDeviceToHost, s));
    // the symbolic tails: the last 32 Ki symbols of each piece's ring, as two 32 KiB byte halves
    std::vector<PpgGather> g(2 * np);
    HIPCHK(hipStreamSynchronize(s));
    clk.mark("f.pass1");
    for (size_t q = 0; q < np; q++) {
        const uint64_t endb = 2 * res[q].produced;
        g[2 * q] = PpgGather{(uint64_t)q * 2 * kPieceRing, (uint64_t)kWin, endb - kWin, 2 * kPieceRing - 1, 0};
        g[2 * q + 1] = PpgGather{(uint64_t)q * 2 * kPieceRing, (uint64_t)kWin, endb, 2 * kPieceRing - 1, 0};
    }
    HIPCHK(grow_buf(F.gat, 2 * np));
    HIPCHK(hipMemcpyAsync(F.gat.p, g.data(), sizeof(PpgGather) * 2 * np, hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_gather(s, F.ring.p, F.ident.p, F.gat.p, F.ta.p, nullptr, nullptr, (int)(2 * np)));
    // the chains: piece j of a chunk is followed when its last block end is piece j+1's start
    std::vector<std::vector<uint32_t>> chain(ch.size());
    // the side point of a chain end is the FIRST block end of its piece with the same output: a
    // sync flush's empty stored block (pigz, Z_SYNC_FLUSH) ends at the same output as the block
    // before it, and the split decode of the piece before a side point stops (pos == len, the
    // end-of-block consumed) at that first end, not past the empty block (a side point there was
    // a DATA_ERROR in ppg_split_merge).  An end that adds no output, or reaches the chunk's end,
    // is walked through but gets no side point (keep = 0).
    struct End { uint64_t bit, out; bool keep; };
    std::vector<std::vector<End>> ends(ch.size());   // chunk-relative output
    for (size_t c = 0; c < ch.size(); c++) {
        uint64_t outc = 0, last_kept = 0;
        for (size_t q = pfirst[c]; q < pfirst[c + 1]; q++) {
            const PpgInflateResult &r = res[q];
            const uint32_t nb = std::min(r.nblocks, jobs[q].blk_cap);
            if (r.status != 0 || nb == 0 || r.last || (r.flags & (PPG_FLAG_BLK_FULL | PPG_FLAG_OVERRUN))) break;
            const PpgBlockEnd *bl = blk.data() + jobs[q].blk_off;
            const uint64_t E = bl[nb - 1].end_bit;
            if (E >= ch[c].bit_end || bl[nb - 1].out_end != r.produced) break;
            uint32_t f = nb - 1;
            while (f > 0 && bl[f - 1].out_end == bl[nb - 1].out_end) f--;
            outc += r.produced;
            const bool keep = outc > last_kept && (int64_t)outc < ch[c].len;
            if (keep) last_kept = outc;
            chain[c].push_back((uint32_t)q);
            ends[c].push_back(End{bl[f].end_bit, outc, keep});
            if (q + 1 >= pfirst[c + 1] || pc[q + 1].start != E) break;   // the next candidate was false
        }
    }
    // histories at the verified block ends, every chain in one launch: W[0] = the Point's window,
    // W[j+1] = T_j(W[j]); the kept ones packed on the device and copied back at once
    size_t wmax = 0;
    for (size_t c = 0; c < ch.size(); c++) wmax = std::max(wmax, chain[c].size() + 1);
    if (wmax < 2) return PPG_OK;
    HIPCHK(grow_buf(F.W, ch.size() * wmax * kWin));
    HIPCHK(grow_buf(F.slots, ch.size() * wmax));
    std::vector<uint32_t> sl_all(ch.size() * wmax, 0);
    std::vector<uint4> cs;
    for (size_t c = 0; c < ch.size(); c++) {
        if (chain[c].empty()) continue;
        std::copy(chain[c].begin(), chain[c].end(), sl_all.begin() + (ptrdiff_t)(c * wmax));
        cs.push_back(uint4{(uint32_t)(c * wmax), (uint32_t)chain[c].size() + 1, ch[c].win, 0});
    }
    HIPCHK(grow_buf(F.chains, cs.size()));
    HIPCHK(hipMemcpyAsync(F.slots.p, sl_all.data(), 4 * sl_all.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(F.chains.p, cs.data(), sizeof(uint4) * cs.size(), hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_resolve_chains(s, F.ta.p, F.slots.p, F.chains.p, (int)cs.size(), dwin, F.W.p));
    const size_t base = sbit.size();
    std::vector<uint32_t> pick;
    for (size_t c = 0; c < ch.size(); c++) {
        bool any = false;
        for (size_t j = 0; j < ends[c].size(); j++) {
            const End &e = ends[c][j];
            if (!e.keep) continue;
            pick.push_back((uint32_t)(c * wmax + j + 1));   // W[j + 1]: the history at the end of chain piece j
            sbit.push_back((int64_t)e.bit);
            sout.push_back(ch[c].out0 + (int64_t)e.out);
            any = true;
        }
        nsplit += any;
    }
    swin.resize((base + pick.size()) * kWin);
    if (!pick.empty()) {
        HIPCHK(grow_buf(F.pick, pick.size()));
        HIPCHK(grow_buf(F.packed, pick.size() * kWin));
        HIPCHK(hipMemcpyAsync(F.pick.p, pick.data(), 4 * pick.size(), hipMemcpyHostToDevice, s));
        HIPCHK(ppg_launch_pick_windows(s, F.W.p, F.pick.p, (int)pick.size(), F.packed.p));
        HIPCHK(hipMemcpyAsync(swin.data() + base * kWin, F.packed.p, pick.size() * kWin, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    clk.mark("f.resolve");
    return PPG_OK;
}

// ---- the materialise path: one symbolic decode per piece instead of two (r05) ----
// A launch of at most kMatMaxChunks chunks of plain indexes (no side points of their own) splits
// each chunk at the inner block starts found on the GPU as find_side_points does, but its pass 1
// covers the WHOLE chunk -- the last piece too, up to the chunk's end -- and keeps every piece's
// symbolic output whole (ppg_inflate_kernel IXF).  A chunk whose chain of block ends is verified
// from its Point to its end gets its pieces' exact starting histories resolved from the symbolic
// tails and is then written out from the symbols (ppg_materialize_kernel, with the fused newline
// census) -- no second decode; any other chunk is decoded whole, one wave, in the same launch.
// A lone 10,000-record chunk: find ~0.5 ms + one symbolic decode of a single deflate block (~4 ms)
// + resolve + materialise, instead of that plus a second decode of the same block.
constexpr int kMatMaxChunks = (int)kMaxBatch;
constexpr uint64_t kMatRatio = 10;        // symbol capacity per compressed byte of a piece (FASTQ: ~4)
// candidate ranges per chunk and their least compressed size: a zlib -6 FASTQ block is ~16 K symbols,
// ~20 KB of gzip, so ranges of ~1/16 chunk (60 KB) held 2-3 block starts of which the finder keeps
// the first, and the slowest piece was several blocks long.  r05 (tools/chunk_latency.py, one box):
// 16 ranges / 48 KiB: T = 1 5.68 ms (pass 1 3.8); 24 / 32: 4.72; 32 / 24: 3.94 (2.36); 48 / 16:
// 2.90 (1.60); 64 / 12: 2.85 (1.61) -- pieces of one block each from 48 on; a 256-chunk launch
// ~45 ms at every setting (the search grows as pass 1 shrinks)
constexpr uint64_t kMatRanges = 48;
constexpr uint64_t kMatMinRange = 16 * 1024;

struct MatPiece {
    uint64_t start, stop;       // bits: piece start, the next piece's start (the chunk's end for the last)
    uint64_t sym_off, cap;      // symbols
};

int find_mat(ChunkSlot &sl, const uint32_t *comp, uint64_t nwords, const uint8_t *dwin, const std::vector<FindChunk> &ch,
             std::vector<uint8_t> &covered, std::vector<std::vector<PpgMatInfo>> &pmi,
             std::vector<std::vector<int64_t>> &pbit, std::vector<std::vector<int64_t>> &pout, PhaseClock &clk) {
    hipStream_t s = sl.s;
    FindScratch &F = sl.fs;
    covered.assign(ch.size(), 0);
    pmi.assign(ch.size(), {});
    pbit.assign(ch.size(), {});
    pout.assign(ch.size(), {});
    std::vector<uint64_t> lo, hi;
    std::vector<size_t> cfirst(ch.size() + 1, 0);
    for (size_t c = 0; c < ch.size(); c++) {
        const uint64_t span = ch[c].bit1 - ch[c].bit0;
        const uint64_t pb = std::max<uint64_t>(8ull * kMatMinRange, span / kMatRanges);
        for (uint64_t a = ch[c].bit0 + pb; a + 8ull * 1024 < ch[c].bit1; a += pb) {
            lo.push_back(a);
            hi.push_back(std::min(a + pb, ch[c].bit1));
        }
        cfirst[c + 1] = lo.size();
    }
    const size_t nc = lo.size();
    std::vector<uint64_t> cand(nc);
    if (nc) {
        HIPCHK(grow_buf(F.lo, nc));
        HIPCHK(grow_buf(F.hi, nc));
        HIPCHK(grow_buf(F.cand, nc));
        HIPCHK(hipMemcpyAsync(F.lo.p, lo.data(), 8 * nc, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(F.hi.p, hi.data(), 8 * nc, hipMemcpyHostToDevice, s));
        HIPCHK(ppg_launch_block_find(s, comp, nwords, F.lo.p, F.hi.p, F.cand.p, (int)nc, find_sub((int)nc)));
        HIPCHK(hipMemcpyAsync(cand.data(), F.cand.p, 8 * nc, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    clk.mark("f.cand");
    // pieces: the Point, the candidates, up to the chunk's end; symbol capacity by compressed size
    std::vector<MatPiece> pc;
    std::vector<size_t> pfirst(ch.size() + 1, 0);
    uint64_t syms = 0;
    for (size_t c = 0; c < ch.size(); c++) {
        std::vector<uint64_t> st{ch[c].bit0};
        for (size_t k = cfirst[c]; k < cfirst[c + 1]; k++)
            if (cand[k] != ~0ull && cand[k] > st.back() && cand[k] < ch[c].bit_end) st.push_back(cand[k]);
        st.push_back(ch[c].bit_end);
        for (size_t j = 0; j + 1 < st.size(); j++) {
            // (at least 192 Ki symbols, ~1.5 zlib -6 FASTQ blocks: a piece whose next candidate is false
            // decodes on to the next real block end, a whole block past a stop that may be only a few
            // KB away; a piece of a typical ~20 KB range gets its 10x anyway, so the floor costs little)
            const uint64_t cap = std::max<uint64_t>(192 * 1024, kMatRatio * ((st[j + 1] - st[j]) / 8 + 64));
            pc.push_back(MatPiece{st[j], st[j + 1], syms, cap});
            syms += cap + 2048;   // flushes may run up to a unit past the capacity check
        }
        pfirst[c + 1] = pc.size();
    }
    const size_t np = pc.size();
    if (!np) return PPG_OK;
    // a repair piece per chunk at most (below): its symbols, block ends and job reserved up front
    // (grow_buf does not keep contents, and a hipFree mid-launch waits for the whole device)
    uint64_t maxcap = 0;
    for (const MatPiece &m : pc) maxcap = std::max(maxcap, m.cap);
    const size_t nrep_cap = ch.size();
    const uint64_t rep_syms = std::max<uint64_t>(4 * (maxcap + 2048), syms / 16);
    std::vector<PpgInflateJob> jobs(np);
    uint64_t nblk = 0;
    for (size_t q = 0; q < np; q++) {
        PpgInflateJob &J = jobs[q];
        J = PpgInflateJob{};
        J.bit_start = pc[q].start;
        J.bit_limit = std::max<uint64_t>(pc[q].stop, 0);
        J.out_off = pc[q].sym_off;
        J.out_len = pc[q].cap;
        J.expect_end = ~0ull;
        J.stop_bit = pc[q].stop;
        J.blk_off = (uint32_t)nblk;
        J.blk_cap = (uint32_t)((pc[q].stop - pc[q].start) / 8 / 2048 + 64);
        nblk += J.blk_cap;
    }
    const uint64_t rep_blk = 64 * nrep_cap + rep_syms / (kMatRatio * 2048) + 64;
    // the piece may read up to its chunk's slice end (the last block of a non-final piece ends past
    // its stop when the next candidate was false)
    for (size_t c = 0; c < ch.size(); c++)
        for (size_t q = pfirst[c]; q < pfirst[c + 1]; q++) jobs[q].bit_limit = ch[c].bit1;
    HIPCHK(grow_buf(F.jobs, np + nrep_cap));
    HIPCHK(grow_buf(F.res, np + nrep_cap));
    GROW_OR_SKIP(F.blk, (size_t)(nblk + rep_blk));
    GROW_OR_SKIP(F.sym, (size_t)(syms + rep_syms) + 64);
    GROW_OR_SKIP(F.ta, (np + nrep_cap) * 2 * kWin);
    clk.mark("f.grow");
    if (!F.ident.p) {   // u16 0..32767: position p < 0 of a piece is history symbol 32768 + p
        std::vector<uint16_t> id(kWin);
        for (int i = 0; i < kWin; i++) id[(size_t)i] = (uint16_t)i;
        HIPCHK(F.ident.alloc(2 * kWin));
        HIPCHK(hipMemcpyAsync(F.ident.p, id.data(), 2 * kWin, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(F.jobs.p, jobs.data(), sizeof(PpgInflateJob) * np, hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_inflate_ixf(s, comp, nwords, F.jobs.p, F.ident.p, (uint8_t *)F.sym.p, F.res.p, F.blk.p, (int)np));
    std::vector<PpgInflateResult> res(np);
    std::vector<PpgBlockEnd> blk((size_t)nblk);
    HIPCHK(hipMemcpyAsync(res.data(), F.res.p, sizeof(PpgInflateResult) * np, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(blk.data(), F.blk.p, sizeof(PpgBlockEnd) * nblk, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    clk.mark("f.pass1");
    // a chunk is covered when its pieces chain from its Point to its end: each piece's last block
    // end is where the chain's next piece starts -- normally the next candidate; after a false
    // candidate (its piece fails, or the piece before it decodes on to the next real block end) the
    // first later piece that starts there, the false ones skipped (r05: ~0.6% of chunks at 48
    // ranges fell back to a one-wave decode of ~45 ms) --, the chain's last piece ends exactly at
    // the chunk's end (or with the final block, for the file's last chunk), and their outputs add up.
    // Two more cases chain (r05: 2 chunks in 1,024 were still left to the one-wave decode):
    //  - the real block start after a false candidate is no candidate at all (the finder keeps one
    //    per range): a repair piece from that block end to the next good piece's start, decoded in
    //    a second, small pass 1;
    //  - an index's last chunk, whose end is known only as its slice's last byte (no R-E5 end check:
    //    expect_end ~0): its last piece ends a block inside that byte, with every byte of the chunk,
    //    and decodes on into a next block header the slice does not hold, failing -- the piece is
    //    taken up to that block end (r05: index chunk 1023 of the bench's per-chunk legs).
    std::vector<size_t> wbase(ch.size(), 0);
    std::vector<std::vector<uint32_t>> chain(ch.size());
    std::vector<uint64_t> E(np, 0);
    std::vector<uint8_t> cut(np, 0);                      // last pieces taken up to a block end in the slice's last byte
    std::vector<std::vector<uint32_t>> reps(ch.size());   // each chunk's repair pieces (indexes >= np)
    struct Repair {
        size_t c;
        uint64_t start, stop;
    };
    std::vector<Repair> want;
    // chunk c's chain; 0 when covered, else why not (PPG_CHUNK_VERBOSE)
    auto walk = [&](size_t c, bool may_repair) -> int {
        chain[c].clear();
        uint64_t tot = 0;
        size_t q = pfirst[c];
        for (;;) {
            PpgInflateResult &r = res[q];
            const uint32_t nb = std::min(r.nblocks, jobs[q].blk_cap);
            if (r.status != 0 && nb > 0 && ch[c].bit_end == ch[c].bit1) {   // an index's last chunk
                const PpgBlockEnd &e = blk[jobs[q].blk_off + nb - 1];
                if (e.end_bit <= ch[c].bit_end && ch[c].bit_end - e.end_bit < 8 &&
                    tot + e.out_end == (uint64_t)ch[c].len && e.out_end <= jobs[q].out_len) {
                    r.status = 0;
                    r.flags = 0;
                    r.produced = e.out_end;
                    r.nblocks = nb;
                    r.last = 0;
                    cut[q] = 1;
                }
            }
            if (r.status != 0 || nb == 0 || (r.flags & (PPG_FLAG_BLK_FULL | PPG_FLAG_OVERRUN)))
                return r.status != 0 ? 1 : nb == 0 ? 2 : (r.flags & PPG_FLAG_BLK_FULL) ? 3 : 4;
            const PpgBlockEnd &e = blk[jobs[q].blk_off + nb - 1];
            if (e.out_end != r.produced) return 5;
            E[q] = e.end_bit;
            chain[c].push_back((uint32_t)q);
            tot += r.produced;
            if (e.end_bit == ch[c].bit_end || cut[q] || (r.last && ch[c].bit_end == ch[c].bit1))
                return (int64_t)tot == ch[c].len ? 0 : 9;
            if (r.last) return 6;
            size_t nx = q < np ? q + 1 : pfirst[c];   // the piece that starts at this end
            while (nx < pfirst[c + 1] && pc[nx].start < e.end_bit) nx++;
            if (nx < pfirst[c + 1] && pc[nx].start == e.end_bit) {
                q = nx;
                continue;
            }
            size_t rq = ~(size_t)0;
            for (uint32_t x : reps[c])
                if (pc[x].start == e.end_bit) rq = x;
            if (rq != ~(size_t)0) {
                q = rq;
                continue;
            }
            if (may_repair) {   // up to the next piece that decoded, or the chunk's end
                while (nx < pfirst[c + 1] && res[nx].status != 0) nx++;
                want.push_back(Repair{c, e.end_bit, nx < pfirst[c + 1] ? pc[nx].start : ch[c].bit_end});
            }
            return 7;
        }
    };
    std::vector<int> why(ch.size(), 0);
    for (size_t c = 0; c < ch.size(); c++) why[c] = walk(c, true);
    if (!want.empty()) {   // the repair pass
        uint64_t rs = syms, rb = nblk;
        std::vector<size_t> rc;
        for (const Repair &w : want) {
            const uint64_t cap = std::max<uint64_t>(192 * 1024, kMatRatio * ((w.stop - w.start) / 8 + 64));
            const uint32_t bc = (uint32_t)((w.stop - w.start) / 8 / 2048 + 64);
            if (w.stop <= w.start || rs + cap + 2048 > syms + rep_syms || rb + bc > nblk + rep_blk) continue;
            PpgInflateJob J{};
            J.bit_start = w.start;
            J.bit_limit = ch[w.c].bit1;
            J.out_off = rs;
            J.out_len = cap;
            J.expect_end = ~0ull;
            J.stop_bit = w.stop;
            J.blk_off = (uint32_t)rb;
            J.blk_cap = bc;
            reps[w.c].push_back((uint32_t)pc.size());
            pc.push_back(MatPiece{w.start, w.stop, rs, cap});
            jobs.push_back(J);
            rc.push_back(w.c);
            rs += cap + 2048;
            rb += bc;
        }
        const size_t nr = pc.size() - np;
        if (nr) {
            res.resize(np + nr);
            blk.resize((size_t)rb);
            E.resize(np + nr, 0);
            cut.resize(np + nr, 0);
            HIPCHK(hipMemcpyAsync(F.jobs.p + np, jobs.data() + np, sizeof(PpgInflateJob) * nr, hipMemcpyHostToDevice, s));
            HIPCHK(ppg_launch_inflate_ixf(s, comp, nwords, F.jobs.p + np, F.ident.p, (uint8_t *)F.sym.p, F.res.p + np,
                                          F.blk.p, (int)nr));
            HIPCHK(hipMemcpyAsync(res.data() + np, F.res.p + np, sizeof(PpgInflateResult) * nr, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(blk.data() + nblk, F.blk.p + nblk, sizeof(PpgBlockEnd) * (rb - nblk),
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            std::sort(rc.begin(), rc.end());
            rc.erase(std::unique(rc.begin(), rc.end()), rc.end());
            for (size_t c : rc) why[c] = walk(c, false);
        }
        clk.mark("f.repair");
    }
    const size_t nt = pc.size();
    size_t nw = 0;
    for (size_t c = 0; c < ch.size(); c++) {
        const bool ok = why[c] == 0;
        if (!ok && clk.on) {
            fprintf(stderr, "PPG_CHUNK not covered: chunk %zu reason %d after %zu chained of %zu pieces\n", c, why[c],
                    chain[c].size(), pfirst[c + 1] - pfirst[c]);
            for (size_t x = pfirst[c]; x < pfirst[c + 1]; x++) {
                const PpgInflateResult &r = res[x];
                const uint32_t nb = std::min(r.nblocks, jobs[x].blk_cap);
                fprintf(stderr, "  piece %zu bits [%llu,%llu) chunk [%llu,%llu) cap %llu: status %d flags %u produced %llu "
                        "blocks %u last_end %llu\n", x - pfirst[c], (unsigned long long)pc[x].start,
                        (unsigned long long)pc[x].stop, (unsigned long long)ch[c].bit0, (unsigned long long)ch[c].bit_end,
                        (unsigned long long)pc[x].cap, (int)r.status, (unsigned)r.flags, (unsigned long long)r.produced, nb,
                        nb ? (unsigned long long)blk[jobs[x].blk_off + nb - 1].end_bit : 0ull);
            }
        }
        covered[c] = ok;
        if (ok) {
            wbase[c] = nw;
            nw += chain[c].size();
        }
    }
    if (!nw) return PPG_OK;
    // symbolic tails (the last 32 Ki symbols of each piece, as two 32 KiB byte halves), then every
    // covered chunk's starting histories: W[0] = the Point's window, W[j+1] = T_j(W[j])
    std::vector<PpgGather> g(2 * nt);
    for (size_t q = 0; q < nt; q++) {
        const uint64_t endb = 2 * res[q].produced, base = 2 * pc[q].sym_off;
        g[2 * q] = PpgGather{base, (uint64_t)kWin, endb - kWin, ~0ull, 0};
        g[2 * q + 1] = PpgGather{base, (uint64_t)kWin, endb, ~0ull, 0};
    }
    HIPCHK(grow_buf(F.gat, 2 * nt));
    HIPCHK(hipMemcpyAsync(F.gat.p, g.data(), sizeof(PpgGather) * 2 * nt, hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_gather(s, (const uint8_t *)F.sym.p, F.ident.p, F.gat.p, F.ta.p, nullptr, nullptr, (int)(2 * nt)));
    GROW_OR_SKIP(F.W, nw * kWin);
    HIPCHK(grow_buf(F.slots, nw));
    std::vector<uint32_t> sl_all(nw, 0);
    std::vector<uint4> cs;
    for (size_t c = 0; c < ch.size(); c++) {
        if (!covered[c]) continue;
        std::copy(chain[c].begin(), chain[c].end(), sl_all.begin() + (ptrdiff_t)wbase[c]);
        cs.push_back(uint4{(uint32_t)wbase[c], (uint32_t)chain[c].size(), ch[c].win, 0});
    }
    HIPCHK(grow_buf(F.chains, cs.size()));
    HIPCHK(hipMemcpyAsync(F.slots.p, sl_all.data(), 4 * nw, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(F.chains.p, cs.data(), sizeof(uint4) * cs.size(), hipMemcpyHostToDevice, s));
    HIPCHK(ppg_launch_resolve_chains(s, F.ta.p, F.slots.p, F.chains.p, (int)cs.size(), dwin, F.W.p));
    // the pieces' materialise info, side points at every later piece's start (launch coordinates)
    for (size_t c = 0; c < ch.size(); c++) {
        if (!covered[c]) continue;
        uint64_t outc = 0, last_end = 0;
        for (size_t j = 0; j < chain[c].size(); j++) {
            const size_t q = chain[c][j];
            last_end = E[q];
            if (res[q].produced == 0) continue;   // an empty piece (a flush block) adds nothing
            if (!pmi[c].empty()) {
                pbit[c].push_back((int64_t)pc[q].start);
                pout[c].push_back(ch[c].out0 + (int64_t)outc);
            }
            PpgMatInfo m{};
            m.sym_off = pc[q].sym_off;
            m.win_off = (wbase[c] + j) * (uint64_t)kWin;
            m.nblocks = res[q].nblocks;
            m.last = res[q].last;
            m.prev = pmi[c].empty() ? 0x100u : 0x1FFu;   // 0x100: the chunk job's own (set below)
            pmi[c].push_back(m);
            outc += res[q].produced;
        }
        // each piece's end: where the next starts, the last one's block end
        for (size_t i = 0; i < pmi[c].size(); i++)
            pmi[c][i].end_bit = i + 1 < pmi[c].size() ? (uint64_t)pbit[c][i] : last_end;
        if (pmi[c].empty()) covered[c] = 0;
    }
    // the H2D sources above (g, sl_all, cs) are pageable vectors that die here: wait for the copies
    // (the phase clock syncs only when verbose)
    HIPCHK(hipStreamSynchronize(s));
    clk.mark("f.resolve", s);
    return PPG_OK;
}

// One launch of the requests `batch` on slot `sl` (the caller holds the slot, not the lock).  Sets
// every request's rc and, for a decoded chunk, where its bytes and descriptors sit in sl.res.
int run_launch(ppg_ctx *ctx, ChunkService &svc, ChunkSlot &sl, std::vector<ChunkReq *> &batch) {
    HIPCHK(hipSetDevice(ctx->device));
    PhaseClock pc;
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
        if (rc == PPG_OK && !side_points_inside(r->ix, r->k)) rc = PPG_ARG_ERROR;
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
    // the materialise path (find_mat) takes launches of plain indexes up to kMatMaxChunks
    bool mat = go.size() <= (size_t)kMatMaxChunks && !getenv("PPG_CHUNK_NO_FIND") && !getenv("PPG_CHUNK_NO_MAT");
    for (size_t i = 0; mat && i < go.size(); i++) mat = go[i]->ix->side_out.empty();
    {   // the shard's buffers with headroom, so launches of growing size do not reallocate each time
        size_t n = go.size(), offb = 0, tot = 0, nsub = 0, nwin = 0;
        for (ChunkReq *r : go) {
            const PpgPoint &from = r->ix->pts[(size_t)r->k], &to = r->ix->pts[(size_t)r->k + 1];
            offb += from.offset.size();
            tot += (size_t)std::max<int64_t>(to.output - from.output, 0);
            const auto &O = r->ix->side_out;
            const size_t own = (size_t)std::max<std::ptrdiff_t>(0, std::lower_bound(O.begin(), O.end(), to.output) -
                                                                      std::upper_bound(O.begin(), O.end(), from.output));
            nsub += own;
            nwin += own;
            if (O.empty() && n <= (size_t)kFindMaxChunks) {
                nsub += kMatRanges;   // the block search's pieces at most
                // side windows: the materialise path fills none (its pieces start from resolved
                // histories, not dictionaries); find_side_points at most 15 per chunk (ADVICE r05:
                // 48 windows of 32 KiB per chunk were reserved and never written, ~400 MB per slot)
                if (!mat) nwin += 16;
            }
        }
        ppg_shard *sh = sl.sh;
        HIPCHK(grow_buf(sh->jobs, n));
        HIPCHK(grow_buf(sh->dicts, (n + nwin) * kWin));
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
    {   // the slices, the alignment gaps and the 256-B tail zeroed (the kernels read whole words past a slice)
        std::vector<Span> cp;
        for (size_t i = 0; i < go.size(); i++) {
            const size_t end = (size_t)at[i] + (size_t)go[i]->slice_len;
            memset(sl.in.p + end, 0, (i + 1 < go.size() ? (size_t)at[i + 1] : comp_len + 256) - end);
            cp.push_back(Span{sl.in.p + at[i], go[i]->slice, (size_t)go[i]->slice_len});
        }
        parallel_copy(cp);
    }
    HIPCHK(hipMemcpyAsync(sl.comp.p, sl.in.p, comp_len + 256, hipMemcpyHostToDevice, sl.s));
    ppg_shard *sh = sl.sh;
    pc.mark("h2d", sl.s);
    int rc = shard_prepare_specs(sh, spec.data(), (int32_t)go.size(), sl.comp.p, (int64_t)comp_len, 0, sl.s, nullptr);
    if (rc != PPG_OK) return rc;
    pc.mark("prepare");
    if (mat) {   // the materialise path (find_mat above)
        std::vector<FindChunk> find;
        for (size_t i = 0; i < go.size(); i++) {
            const PpgInflateJob &J = sh->h_jobs[i];
            find.push_back(FindChunk{J.bit_start, J.bit_limit, J.expect_end != ~0ull ? J.expect_end : J.bit_limit,
                                     sh->h_pout[i], (int64_t)J.out_len, (uint32_t)i});
        }
        std::vector<uint8_t> covered;
        std::vector<std::vector<PpgMatInfo>> pmi;
        std::vector<std::vector<int64_t>> pbit, pout;
        rc = find_mat(sl, (const uint32_t *)sl.comp.p, sh->nwords, sh->dicts.p, find, covered, pmi, pbit, pout, pc);
        if (rc == PPG_MEM_ERROR) {   // no room for the search's scratch: every chunk decoded whole
            covered.assign(go.size(), 0);
            rc = PPG_OK;
        }
        if (rc != PPG_OK) return rc;
        std::vector<int64_t> sbit, sout;
        size_t ncov = 0;
        for (size_t i = 0; i < go.size(); i++) {
            if (!covered[i]) continue;
            ncov++;
            sbit.insert(sbit.end(), pbit[i].begin(), pbit[i].end());
            sout.insert(sout.end(), pout[i].begin(), pout[i].end());
        }
        svc.found_chunks += (int64_t)ncov;
        svc.found_points += (int64_t)sbit.size();
        if (!sbit.empty()) {   // (chunks of one piece each only: decoded as usual)
            rc = shard_set_split_impl(sh, (int32_t)sbit.size(), sbit.data(), sout.data(), nullptr, false);
            if (rc != PPG_OK) return rc;
            // launch order: the chunks decoded whole first (longest first), then the materialised pieces
            const auto &X = sh->h_sidx;
            const size_t ns = X[go.size()];
            std::vector<uint32_t> order;
            for (size_t i = 0; i < go.size(); i++)
                if (!covered[i]) order.push_back(X[i]);
            std::stable_sort(order.begin(), order.end(),
                             [&](uint32_t a, uint32_t b) { return sh->h_sjobs[a].out_len > sh->h_sjobs[b].out_len; });
            const uint32_t ndec = (uint32_t)order.size();
            std::vector<PpgMatInfo> lmi;
            for (size_t i = 0; i < go.size(); i++) {
                if (!covered[i]) continue;
                if (X[i + 1] - X[i] != pmi[i].size()) return PPG_DATA_ERROR;   // side points and pieces disagree
                for (uint32_t j = X[i]; j < X[i + 1]; j++) {
                    order.push_back(j);
                    PpgMatInfo m = pmi[i][j - X[i]];
                    if (m.prev == 0x100u) m.prev = sh->h_sjobs[j].prev_byte;   // the chunk's first piece
                    lmi.push_back(m);
                }
            }
            std::vector<PpgInflateJob> lj(ns);
            std::vector<uint32_t> inv(ns);
            for (size_t q = 0; q < ns; q++) {
                lj[q] = sh->h_sjobs[order[q]];
                inv[order[q]] = (uint32_t)q;
            }
            HIPCHK(grow_buf(sh->ljobs, ns));   // (grow-only with headroom: a hipFree waits for the
            HIPCHK(grow_buf(sh->linv, ns));    // whole device, every other slot's launch included)
            HIPCHK(grow_buf(sl.fs.mi, lmi.size()));
            HIPCHK(hipMemcpyAsync(sh->ljobs.p, lj.data(), sizeof(PpgInflateJob) * ns, hipMemcpyHostToDevice, sl.s));
            HIPCHK(hipMemcpyAsync(sh->linv.p, inv.data(), 4 * ns, hipMemcpyHostToDevice, sl.s));
            HIPCHK(hipMemcpyAsync(sl.fs.mi.p, lmi.data(), sizeof(PpgMatInfo) * lmi.size(), hipMemcpyHostToDevice, sl.s));
            sh->lpt = true;
            sh->mat_first = ndec;
            sh->mat_n = (uint32_t)lmi.size();
            sh->mat_sym = sl.fs.sym.p;
            sh->mat_win = sl.fs.W.p;
            sh->mat_info = sl.fs.mi.p;
            HIPCHK(hipStreamSynchronize(sl.s));   // the host staging vectors die here
        }
        pc.mark("split");
    } else {   // side points of the chunks that have them (the index's, shifted into this launch); the
        // others' found on the GPU when the launch is too small to fill it
        std::vector<int64_t> sbit, sout;
        ByteVec swin;
        std::vector<FindChunk> find;
        const bool findable = go.size() <= (size_t)kFindMaxChunks && !getenv("PPG_CHUNK_NO_FIND");
        for (size_t i = 0; i < go.size(); i++) {
            if (!go[i]->ix->side_out.empty()) {
                side_points_of(go[i]->ix, go[i]->k, sh->h_jobs[i].bit_start, sh->h_pout[i], sbit, sout, swin);
            } else if (findable && sh->h_jobs[i].out_len > 0) {
                // sorted by output with the others: flush the found ones in launch order
                const PpgInflateJob &J = sh->h_jobs[i];
                find.push_back(FindChunk{J.bit_start, J.bit_limit, J.expect_end != ~0ull ? J.expect_end : J.bit_limit,
                                         sh->h_pout[i], (int64_t)J.out_len, (uint32_t)i});
            }
            if (!find.empty() && (i + 1 == go.size() || !go[i + 1]->ix->side_out.empty())) {
                const size_t before = sbit.size();
                int64_t nsplit = 0;
                rc = find_side_points(sl, (const uint32_t *)sl.comp.p, sh->nwords, sh->dicts.p, find, sbit, sout, swin, nsplit, pc);
                if (rc != PPG_OK) return rc;
                svc.found_chunks += nsplit;
                svc.found_points += (int64_t)(sbit.size() - before);
                find.clear();
            }
        }
        pc.mark("find");
        if (!sbit.empty()) {
            rc = ppg_shard_set_split(sh, (int32_t)sbit.size(), sbit.data(), sout.data(), swin.data());
            if (rc != PPG_OK) return rc;
        }
        pc.mark("split");
    }
    shard_reset(sh);
    float total_ms = 0;
    rc = batch_launch(sh, 0, sh->n);
    if (rc == PPG_OK) rc = batch_collect(sh, 0, sh->n, total_ms);
    if (sh->mat_n) {   // the slot's shard is reused: the next launch sets its own split
        sh->mat_n = 0;
        sh->nsub = 0;
        sh->lpt = false;
    }
    if (rc != PPG_OK) return rc;
    pc.mark("decode");
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
    pc.mark("d2h");
    pc.dump(go.size(), (int)(&sl - svc.slot));
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

namespace {

// a free slot (not decoding, nobody copying out of it), or -1
int free_slot(const ChunkService &svc) {
    for (int i = 0; i < kChunkSlots; i++)
        if (!svc.slot[i].busy && svc.slot[i].readers == 0) return i;
    return -1;
}

// the batching rule: a launch when nothing decodes, or a full enough queue beside a running one
bool may_lead(const ChunkService &svc) {
    return !svc.pending.empty() && (svc.in_flight == 0 || svc.pending.size() >= kMinSecond);
}

using Svc = ChunkService;

// async requests' results into the buffers given at submit, all at once (up to 8 threads); their
// wait() then only hands back the status and counts
int copy_async_results(const std::vector<ChunkReq *> &reqs) {
    try {
        std::vector<Span> cp;
        for (ChunkReq *r : reqs)
            r->fin_rc = result_spans(*r, r->out, r->out_cap, r->recs, r->rec_cap, r->fin_len, r->fin_nrec, cp);
        parallel_copy(cp, true);
    } catch (...) {
        return PPG_MEM_ERROR;
    }
    for (ChunkReq *r : reqs) r->copied = true;
    return PPG_OK;
}

// the copier thread (started by the first launch with async requests): drains the copy queue, then
// exits once the service stops
void copier_loop(ChunkService *svc) {
    std::unique_lock<std::mutex> lk(svc->mu);
    for (;;) {
        // (a launch still in flight may queue one more task: exit only after it)
        svc->cv.wait(lk, [&] { return !svc->copies.empty() || (svc->stop && svc->in_flight == 0); });
        if (svc->copies.empty()) return;
        Svc::CopyTask t = std::move(svc->copies.front());
        svc->copies.pop_front();
        lk.unlock();
        PhaseClock clk;
        const int rc = copy_async_results(t.reqs);
        if (clk.on) {
            int64_t b = 0;
            for (ChunkReq *r : t.reqs) b += r->fin_len + 16 * (r->recs ? r->nrec : 0);
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - clk.t0).count();
            fprintf(stderr, "PPG_CHUNK copy of %zu: %.1f MB in %.3f ms (slot %d)\n", t.reqs.size(), b / 1e6, ms, t.slot);
        }
        lk.lock();
        for (ChunkReq *r : t.reqs) {
            if (rc != PPG_OK) r->rc = rc;
            r->done = true;
        }
        svc->slot[t.slot].readers--;
        svc->cv.notify_all();
    }
}

// Lead one launch of the queued requests on slot i (lk held on entry and on return, released
// while the launch runs).  Every request of the batch is marked done; a decoded one holds a reader
// on the slot until its results are copied out.
void lead(ppg_ctx *ctx, ChunkService &svc, std::unique_lock<std::mutex> &lk, int i) {
    const size_t nb = std::min(svc.pending.size(), kMaxBatch);
    std::vector<ChunkReq *> batch(svc.pending.begin(), svc.pending.begin() + (ptrdiff_t)nb);
    svc.pending.erase(svc.pending.begin(), svc.pending.begin() + (ptrdiff_t)nb);
    ChunkSlot &sl = svc.slot[i];
    sl.busy = true;
    svc.in_flight++;
    svc.launches++;
    svc.max_batch = std::max<int64_t>(svc.max_batch, (int64_t)batch.size());
    lk.unlock();
    int rc;
    try {
        rc = run_launch(ctx, svc, sl, batch);
    } catch (const std::bad_alloc &) {   // host vectors: never out through the C ABI, never a stuck slot
        rc = PPG_MEM_ERROR;
    } catch (...) {
        rc = PPG_DEVICE_ERROR;
    }
    lk.lock();
    // async requests go to the copier, which marks them done once their results are in the caller's
    // buffers (the copies of a 256-chunk launch take about as long as the launch: done here, they
    // kept the launcher from leading the next one)
    Svc::CopyTask task{i, {}};
    for (ChunkReq *r : batch) {
        if (rc != PPG_OK) r->rc = rc;
        if (r->rc == PPG_OK && r->async) {
            task.reqs.push_back(r);
            continue;
        }
        if (r->rc == PPG_OK) {
            r->slot = i;
            sl.readers++;
        }
        r->done = true;
    }
    if (!task.reqs.empty()) {
        bool queued = false;
        try {
            if (!svc.copier.joinable()) svc.copier = std::thread(copier_loop, &svc);
            svc.copies.push_back(std::move(task));
            sl.readers++;   // the copier's
            queued = true;
        } catch (...) {
        }
        if (!queued) {   // no copier: copy here, the lock released
            lk.unlock();
            const int crc = copy_async_results(task.reqs);
            lk.lock();
            for (ChunkReq *r : task.reqs) {
                if (crc != PPG_OK) r->rc = crc;
                r->done = true;
            }
        }
    }
    sl.busy = false;
    svc.in_flight--;
    svc.cv.notify_all();
}

// copy a done request's results out of its slot (callers copy in parallel), release the slot
int finish(ChunkService &svc, ChunkReq &req, uint8_t *out, int64_t out_cap, int64_t *produced, uint32_t *recs,
           int64_t rec_cap, int64_t *nrec) {
    if (req.copied) {   // an async request the launcher already copied out
        if (produced) *produced = req.fin_len;
        if (nrec && req.fin_nrec) *nrec = req.nrec;
        return req.fin_rc;
    }
    int rc = req.rc;
    if (rc == PPG_OK) {
        int64_t len = 0;
        bool with_nrec = false;
        std::vector<Span> cp;
        try {
            rc = result_spans(req, out, out_cap, recs, rec_cap, len, with_nrec, cp);
            parallel_copy(cp, true);
        } catch (...) {
            rc = PPG_MEM_ERROR;
        }
        if (produced) *produced = len;
        if (nrec && with_nrec) *nrec = req.nrec;
        std::lock_guard<std::mutex> lk(svc.mu);
        if (--svc.slot[req.slot].readers == 0) svc.cv.notify_all();
    }
    return rc;
}

// the launcher of asynchronous requests: whenever requests are queued and the batching rule allows,
// after letting a burst of submissions settle (a caller queueing hundreds of chunks gets them into
// one launch, not the first few into a launch of their own)
void worker_loop(ChunkService *svc) {
    using namespace std::chrono;
    std::unique_lock<std::mutex> lk(svc->mu);
    for (;;) {
        svc->cv.wait(lk, [&] { return svc->stop || (may_lead(*svc) && free_slot(*svc) >= 0); });
        if (svc->stop) return;
        while (svc->pending.size() < kMaxBatch && steady_clock::now() - svc->last_submit < microseconds(200))
            svc->cv.wait_for(lk, microseconds(100));
        const int i = free_slot(*svc);
        if (i < 0 || !may_lead(*svc)) continue;
        lead(svc->ctx, *svc, lk, i);
    }
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
    svc->cv.notify_all();
    while (!req.done) {
        const int i = free_slot(*svc);
        if (i < 0 || !may_lead(*svc)) {
            svc->cv.wait(lk);
            continue;
        }
        // lead a launch of the queued requests (this one among them, unless another caller took it)
        lead(ctx, *svc, lk, i);
    }
    lk.unlock();
    return finish(*svc, req, out, out_cap, produced, recs, rec_cap, nrec);
}

int ppg_decompress_chunk_submit(ppg_ctx *ctx, const ppg_index *ix, int32_t k, const uint8_t *slice, int64_t slice_len,
                                uint8_t *out, int64_t out_cap, uint32_t *recs, int64_t rec_cap, ppg_chunk_req **req) {
    if (!ctx || !ix || !slice || !req || k < 0 || (size_t)k + 1 >= ix->pts.size() || !ctx->chunks) return PPG_ARG_ERROR;
    ChunkService *svc = ctx->chunks;
    auto *r = new (std::nothrow) ChunkReq{ix, k, slice, slice_len};
    if (!r) return PPG_MEM_ERROR;
    r->async = true;
    r->out = out;
    r->out_cap = out_cap;
    r->recs = recs;
    r->rec_cap = rec_cap;
    {
        std::lock_guard<std::mutex> lk(svc->mu);
        if (!svc->worker[0].joinable()) {
            svc->ctx = ctx;
            try {
                svc->worker[0] = std::thread(worker_loop, svc);
            } catch (...) {
                delete r;
                return PPG_MEM_ERROR;
            }
            for (int w = 1; w < kLaunchers; w++) {   // (more launchers are an optimisation only)
                try {
                    svc->worker[w] = std::thread(worker_loop, svc);
                } catch (...) {
                }
            }
        }
        svc->calls++;
        svc->pending.push_back(r);
        svc->last_submit = std::chrono::steady_clock::now();
    }
    svc->cv.notify_all();
    *req = (ppg_chunk_req *)r;
    return PPG_OK;
}

int ppg_decompress_chunk_wait(ppg_ctx *ctx, ppg_chunk_req *ticket, int64_t *produced, int64_t *nrec) {
    if (!ctx || !ticket || !ctx->chunks) return PPG_ARG_ERROR;
    ChunkService *svc = ctx->chunks;
    ChunkReq *r = (ChunkReq *)ticket;
    {
        std::unique_lock<std::mutex> lk(svc->mu);
        svc->cv.wait(lk, [&] { return r->done; });
    }
    const int rc = finish(*svc, *r, r->out, r->out_cap, produced, r->recs, r->rec_cap, nrec);
    delete r;
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

int ppg_decompress_chunk_split_stats(ppg_ctx *ctx, int64_t *chunks, int64_t *side_points) {
    if (!ctx || !ctx->chunks) return PPG_ARG_ERROR;
    if (chunks) *chunks = ctx->chunks->found_chunks.load();
    if (side_points) *side_points = ctx->chunks->found_points.load();
    return PPG_OK;
}

}  // extern "C"

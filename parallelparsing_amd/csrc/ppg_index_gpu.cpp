// ppg_index_gpu.cpp — CreateIndex on the GPU: the same Points as Core.BuildDeflateIndex
// (Decompressor/Core.cs:14-131; the host restatement is IndexBuilder in ppg_api.cpp).
//
// The reference makes one serial zlib inflate(Z_BLOCK) pass over the member, counting '@' bytes
// and dropping a Point at the first block end after more than chunksize-8 of them.  The Points
// depend only on (a) where the deflate blocks end, (b) how many '@' each block emits, (c) the
// 32 KiB of output before each chosen block end.  All three come out of a block-parallel decode:
//
//   1. finder     the compressed member is cut into pieces of piece_bytes; one wave per piece
//                 finds the first bit where a dynamic-block header zlib would accept starts
//                 (ppg_block_find_kernel).  Piece 0 starts right after the gzip header.
//   2. pass 1     every piece decodes whole blocks from its candidate until a block ends at or
//                 past the next piece's candidate, recording each block end (ppg_inflate_kernel
//                 IX).  Block boundaries do not depend on history bytes, so walking the pieces in
//                 order proves each start: piece j+1 is real iff the (real) piece j ended exactly
//                 there; otherwise piece j+1 is redone from where piece j really ended.  The
//                 history is unknown, so pass 1's output is symbolic, 16 bits per position: a
//                 literal byte, or "a copy of history byte i" (r03; r02 decoded every piece twice,
//                 over two synthetic histories, to tell the two apart).  FASTQ needs this: a
//                 header's "length=150" is copied from the previous record's, a chain that runs
//                 back to the piece's start, so tails depend on the starting history.
//   3. resolve    the exact starting history of every piece, walking the chain of symbolic
//                 tails from the stream start (one 32 KiB gather per piece).
//   4. pass 2     every piece decoded again with its exact history (the DecompressAll kernel);
//                 its tail must reproduce the resolved history of the next piece.
//   5. census     per-block '@' statistics over the exact output (ppg_at_stats_kernel); the host
//                 walks the blocks in order exactly as Core.cs:98-110 does and gathers the 32 KiB
//                 windows of the chosen Points on the GPU (ppg_gather_kernel).
//
// Scope: single-member gzip (the reference's input).  A zlib-wrapped stream, a
// multi-member file or trailing bytes return PPG_UNSUPPORTED (ppg_index_build_file handles them).
// The trailer's ISIZE and CRC-32 are checked as zlib's gzip mode does (Core.cs:30 inflateInit2(47)):
// a mismatch is PPG_DATA_ERROR.  The CRC is computed on the GPU over each pass-2 batch
// (ppg_crc_kernel) and folded on the host (crc_fold below).
#include "ppg_host.h"
#include <zlib.h>
#include <chrono>
#include <cstdlib>
#include <algorithm>
#include <memory>
#include <thread>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

hipError_t ppg_launch_inflate(hipStream_t s, int ring_bits, int lit_bits, const uint32_t *comp, uint64_t nwords,
                              const PpgInflateJob *jobs, const uint8_t *dicts, uint8_t *out, PpgInflateResult *res,
                              int njobs, uint32_t *nls);
hipError_t ppg_launch_inflate_ix(hipStream_t s, const uint32_t *comp, uint64_t nwords, const PpgInflateJob *jobs,
                                 const uint8_t *dicts, uint8_t *out, PpgInflateResult *res, PpgBlockEnd *blk,
                                 int njobs);
hipError_t ppg_launch_block_find(hipStream_t s, const uint32_t *comp, uint64_t nwords, const uint64_t *lo,
                                 const uint64_t *hi, uint64_t *cand, int n, int sub);
hipError_t ppg_launch_gather(hipStream_t s, const uint8_t *out, const uint8_t *dicts, const PpgGather *g, uint8_t *dst,
                             const uint8_t *ref, uint32_t *diff, int n);
hipError_t ppg_launch_at_stats(hipStream_t s, const uint8_t *out, const PpgSpan *spans, PpgAtStats *st, int n);
hipError_t ppg_launch_resolve(hipStream_t s, const uint8_t *ta, const uint8_t *tb, const uint32_t *slots, int np,
                              uint8_t *W, uint16_t *M);
int ppg_resolve_groups(int np);
hipError_t ppg_launch_crc(hipStream_t s, const uint8_t *out, uint64_t n, uint64_t pad, const uint32_t *tabs,
                          uint32_t *seg_raw, uint64_t nseg);
hipError_t ppg_launch_pack_blocks(hipStream_t s, const PpgBlockEnd *blk, const PpgInflateJob *jobs,
                                  const PpgInflateResult *res, const uint64_t *pre, PpgBlockEnd *dense, int n);

namespace {

constexpr uint64_t kRing = 65536;       // pass-1 output ring per piece (IX_RING_BYTES)
constexpr int64_t kMaxRun = kWin;       // at most 32768 bytes since the last '@'
constexpr uint64_t kPass2Cap = 96ull << 30;   // default pass-2 output buffer
constexpr uint32_t kSpare = 256;        // pass-1 slots for speculative redos of false starts

// spare slots: kSpare, or PPG_IX_SPARES (tests: 0 sends every false start down the serial redo)
uint32_t spare_slots() {
    const char *e = getenv("PPG_IX_SPARES");
    return e && *e ? (uint32_t)std::min(atol(e) < 0 ? 0L : atol(e), 1L << 16) : kSpare;
}

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// device -> pageable host through the ctx's pinned staging buffer (two halves: the copy engine
// fills one while host threads fan the other out).  A direct pageable copy of a batch's windows
// (~860 MB) ran at ~10 GB/s, and at ~0.5 GB/s when the index's freshly grown pages were first
// touched by it (r03: 1.6 s in one run of two).
int copy_d2h_staged(ppg_ctx *ctx, hipStream_t s, uint8_t *dst, const uint8_t *src, size_t n) {
    constexpr size_t kHalf = 128ull << 20;
    constexpr int kThreads = 8;
    if (!n) return PPG_OK;
    if (!ctx->stage) {
        HIPCHK(hipHostMalloc((void **)&ctx->stage, 2 * kHalf, hipHostMallocDefault));
        ctx->stage_n = 2 * kHalf;
    }
    auto fan_out = [&](uint8_t *d, const uint8_t *h, size_t m) {
        std::thread th[kThreads];
        const size_t part = (m + kThreads - 1) / kThreads;
        for (int t = 0; t < kThreads; t++) {
            const size_t a = std::min(m, t * part), b = std::min(m, a + part);
            th[t] = std::thread([=] { if (b > a) memcpy(d + a, h + a, b - a); });
        }
        for (auto &x : th) x.join();
    };
    size_t prev_o = 0, prev_m = 0;
    int half = 0;
    for (size_t o = 0; o < n; o += kHalf, half ^= 1) {
        const size_t m = std::min(kHalf, n - o);
        HIPCHK(hipMemcpyAsync(ctx->stage + half * kHalf, src + o, m, hipMemcpyDeviceToHost, s));
        if (prev_m) fan_out(dst + prev_o, ctx->stage + (half ^ 1) * kHalf, prev_m);   // while the copy runs
        HIPCHK(hipStreamSynchronize(s));
        prev_o = o;
        prev_m = m;
    }
    fan_out(dst + prev_o, ctx->stage + (half ^ 1) * kHalf, prev_m);
    return PPG_OK;
}

// Pages of [p, p + n) faulted in ahead of a bulk copy into them (huge pages where the kernel
// allows): a first touch by the copy itself cost ~60 ms per 860 MB of windows (r03)
void prefault(uint8_t *p, size_t n) {
    const uintptr_t a = ((uintptr_t)p + 4095) & ~(uintptr_t)4095, z = ((uintptr_t)p + n) & ~(uintptr_t)4095;
    if (z <= a) return;
    (void)madvise((void *)a, z - a, MADV_HUGEPAGE);
#ifdef MADV_POPULATE_WRITE
    (void)madvise((void *)a, z - a, MADV_POPULATE_WRITE);
#endif
}

// capacity for `need` elements, reserved as need x max(scale, 1.5) when it has to grow
template <class V>
void grow(V &v, size_t need, double scale) {
    if (need <= v.capacity()) return;
    v.reserve(std::max<size_t>(need, (size_t)((double)need * std::max(scale, 1.5))));
}

// RFC 1952 member header length, or -1 (not a gzip member this path handles)
int64_t gzip_header_len(const uint8_t *h, int64_t n) {
    if (n < 10 || h[0] != 31 || h[1] != 139 || h[2] != 8) return -1;
    const int flg = h[3];
    if (flg & 0xE0) return -1;
    int64_t p = 10;
    if (flg & 4) {                      // FEXTRA
        if (p + 2 > n) return -1;
        p += 2 + (int64_t)(h[p] | (h[p + 1] << 8));
    }
    for (int f : {8, 16}) {             // FNAME, FCOMMENT: zero-terminated
        if (!(flg & f)) continue;
        while (p < n && h[p]) p++;
        if (p >= n) return -1;
        p++;
    }
    if (flg & 2) p += 2;                // FHCRC
    return p <= n ? p : -1;
}

// CRC-32 register algebra for ppg_crc_kernel (see ppg_index.hip): Z(c, n) = the register after n
// zero bytes, linear in c, = zlib's crc32_combine(c, 0, n).  Tables give Z(., n) bytewise.
struct CrcTables {
    uint32_t dev[2048];                 // [0,1024): slicing-by-4 byte tables, [1024,2048): Z(., kCrcSub)
    uint32_t seg[1024];                 // Z(., kCrcSeg), for the host fold
    CrcTables() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1)));
            dev[i] = c;
        }
        for (int t = 1; t < 4; t++)
            for (uint32_t i = 0; i < 256; i++) dev[256 * t + i] = (dev[256 * (t - 1) + i] >> 8) ^ dev[dev[256 * (t - 1) + i] & 255];
        for (int k = 0; k < 4; k++)
            for (uint32_t b = 0; b < 256; b++) {
                dev[1024 + 256 * k + b] = (uint32_t)crc32_combine(b << (8 * k), 0, kCrcSub);
                seg[256 * k + b] = (uint32_t)crc32_combine(b << (8 * k), 0, kCrcSeg);
            }
    }
    uint32_t zseg(uint32_t r) const {
        return seg[r & 255] ^ seg[256 + ((r >> 8) & 255)] ^ seg[512 + ((r >> 16) & 255)] ^ seg[768 + (r >> 24)];
    }
};

struct Piece {
    uint32_t slot;                      // pass-1 job / ring / tail slot
    uint64_t start;                     // absolute bit of the piece's first block header
};

struct Builder {
    ppg_ctx *ctx;
    hipStream_t s;
    const uint32_t *comp;
    uint64_t nwords;
    int64_t len;
    uint32_t chunksize;
    double *stat;                       // ctx->ix_stats

    // pass 1
    std::vector<PpgInflateJob> hjobs;
    std::vector<PpgInflateResult> hres;
    // host block lists, dense: slot q's at hblk[hpos[q]] (a re-run slot's newer list is appended);
    // addressed by the device's blk_off instead, the 29M-entry array was page-faulted in for a
    // few entries per piece (r03: 84 ms of zero fill, then 45 ms of faults)
    std::vector<PpgBlockEnd> hblk;
    std::vector<uint64_t> hpos;
    DevBuf<PpgBlockEnd> blk, bigblk;   // block lists of pass-1 job q at blk_off (bigblk: a piece alone)
    DevBuf<uint8_t> ring;               // 64 Ki 16-bit symbols of output ring per slot
    DevBuf<uint8_t> ident;              // u16 0..32767: the history symbols, for tails of short pieces
    DevBuf<uint8_t> ta;                 // symbolic tail (32 Ki u16) of pass-1 job q at q * 64 KiB
    DevBuf<PpgGather> gat;
    DevBuf<uint32_t> diff;
    DevBuf<uint64_t> dpre;
    DevBuf<PpgBlockEnd> dense;

    uint32_t nslots = 0;                // pieces + spare slots for speculative redos
    DevBuf<PpgInflateJob> jst;          // staged jobs of a pass-1 launch
    DevBuf<PpgInflateResult> rst;

    // pass-1 decode of job slots `which` (ascending) in one launch, 16-bit symbolic output into
    // ring slot q; refreshes their results, block lists and symbolic tails
    int run_pass1(const std::vector<uint32_t> &which, bool big) {
        if (which.empty()) return PPG_OK;
        const size_t n = which.size();
        std::vector<PpgInflateJob> st(n);
        for (size_t i = 0; i < n; i++) {
            st[i] = hjobs[which[i]];
            st[i].dict_off = 0;
        }
        HIPCHK(jst.alloc(n));
        HIPCHK(rst.alloc(n));
        HIPCHK(hipMemcpyAsync(jst.p, st.data(), sizeof(PpgInflateJob) * n, hipMemcpyHostToDevice, s));
        const auto tk = Clock::now();
        HIPCHK(ppg_launch_inflate_ix(s, comp, nwords, jst.p, ident.p, ring.p, rst.p, big ? bigblk.p : blk.p, (int)n));
        std::vector<PpgInflateResult> r(n);
        HIPCHK(hipMemcpyAsync(r.data(), rst.p, sizeof(PpgInflateResult) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const double t_kern = ms_since(tk);
        for (size_t i = 0; i < n; i++) hres[which[i]] = r[i];
        // the tails: the last 32 Ki symbols (64 KiB) of each ring, gathered as two 32 KiB byte
        // halves; a position before the piece's start is history symbol 32768 + p (ident table)
        std::vector<PpgGather> g(2 * n);
        for (size_t i = 0; i < n; i++) {
            const uint32_t q = which[i];
            const uint64_t endb = 2 * hres[q].produced;   // byte position of the ring's end
            g[2 * i] = PpgGather{(uint64_t)q * 2 * kRing, (uint64_t)kWin, endb - kWin, 2 * kRing - 1, 0};
            g[2 * i + 1] = PpgGather{(uint64_t)q * 2 * kRing, (uint64_t)kWin, endb, 2 * kRing - 1, 0};
        }
        HIPCHK(gat.alloc(g.size()));
        HIPCHK(hipMemcpyAsync(gat.p, g.data(), sizeof(PpgGather) * g.size(), hipMemcpyHostToDevice, s));
        for (size_t i = 0; i < n;) {   // one gather per contiguous run of slots
            size_t e = i + 1;
            while (e < n && which[e] == which[e - 1] + 1) e++;
            HIPCHK(ppg_launch_gather(s, ring.p, ident.p, gat.p + 2 * i, ta.p + (uint64_t)which[i] * 2 * kWin, nullptr,
                                     nullptr, (int)(2 * (e - i))));
            i = e;
        }
        if (big) {
            const uint32_t q = which[0];
            const uint32_t nb = std::min(hres[q].nblocks, hjobs[q].blk_cap);
            hblk_big.assign(nb, PpgBlockEnd{0, 0});
            if (nb) HIPCHK(hipMemcpyAsync(hblk_big.data(), bigblk.p, sizeof(PpgBlockEnd) * nb, hipMemcpyDeviceToHost, s));
        } else {
            // pack run A's block lists densely on the device, one copy back
            std::vector<uint64_t> pre(n + 1, 0);
            for (size_t i = 0; i < n; i++) pre[i + 1] = pre[i] + std::min(hres[which[i]].nblocks, hjobs[which[i]].blk_cap);
            HIPCHK(dpre.alloc(pre.size()));
            HIPCHK(dense.alloc(pre.back() + 1));
            HIPCHK(hipMemcpyAsync(dpre.p, pre.data(), 8 * pre.size(), hipMemcpyHostToDevice, s));
            HIPCHK(ppg_launch_pack_blocks(s, blk.p, jst.p, rst.p, dpre.p, dense.p, (int)n));
            const size_t h0 = hblk.size();
            hblk.resize(h0 + pre.back());
            if (pre.back())
                HIPCHK(hipMemcpyAsync(hblk.data() + h0, dense.p, sizeof(PpgBlockEnd) * pre.back(), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            for (size_t i = 0; i < n; i++) hpos[which[i]] = h0 + pre[i];
        }
        HIPCHK(hipStreamSynchronize(s));
        if (getenv("PPG_IX_VERBOSE"))
            fprintf(stderr, "[ix] pass 1 run of %zu jobs: kernel %.1f ms, tails + blocks %.1f\n", n, t_kern,
                    ms_since(tk) - t_kern);
        return PPG_OK;
    }
    std::vector<PpgBlockEnd> hblk_big;
    std::vector<std::vector<PpgBlockEnd>> own_blocks;   // per slot, when decoded into bigblk

    const PpgBlockEnd *blocks(uint32_t q, uint32_t &nb) const {
        nb = hres[q].nblocks;
        if (!own_blocks[q].empty()) return own_blocks[q].data();
        return hblk.data() + hpos[q];
    }
};

}  // namespace

static int build_index_gpu(ppg_ctx *ctx, const uint8_t *dcomp, int64_t len, const uint8_t *head, int64_t head_n,
                           const uint8_t trailer[8], uint32_t chunksize, int64_t piece_bytes, int64_t out_capacity,
                           int64_t side_bytes, ppg_index &ix) {
    const auto t_all = Clock::now();
    double *stat = ctx->ix_stats;
    std::fill(stat, stat + kIxStats, 0.0);
    const int64_t hl = gzip_header_len(head, head_n);
    if (hl < 0 || len < hl + 8 + 1) return PPG_UNSUPPORTED;
    Builder B;
    B.ctx = ctx;
    B.s = ctx->stream;
    B.comp = (const uint32_t *)dcomp;
    B.nwords = (uint64_t)(len + 3) / 4;
    B.len = len;
    B.chunksize = chunksize;
    B.stat = stat;
    hipStream_t s = B.s;
    const uint64_t d0 = 8ull * (uint64_t)hl;
    const uint64_t end_bits = 8ull * (uint64_t)(len - 8);   // no block header starts in the trailer
    // default ~65k pieces (768 KiB for a 50 GB member: 3.41 s vs 3.72 s at 16k pieces, r02 --ix-piece-kib
    // sweep -- pass 2's batches hold several generations of waves; smaller pieces cost more setup)
    if (piece_bytes <= 0) {
        piece_bytes = std::min<int64_t>(4 << 20, std::max<int64_t>(256 << 10, len / 65536));
        // a caller-sized pass-2 buffer holds ~4 output bytes per compressed byte: at most
        // capacity / 32768 per piece keeps ~8k pieces (a generation of waves) per batch
        // (16 GiB: 512 KiB pieces, 2.18 -> 2.02 s for the 50 GB member, r03 v5 sweep)
        if (out_capacity > 0) piece_bytes = std::max<int64_t>(256 << 10, std::min<int64_t>(piece_bytes, out_capacity / 32768));
    }
    const uint64_t pbits = 8ull * (uint64_t)piece_bytes;

    // ---- 1. candidate block starts ----
    auto t = Clock::now();
    std::vector<uint64_t> lo, hi;
    for (uint64_t a = d0 + pbits; a < end_bits; a += pbits) {
        lo.push_back(a);
        hi.push_back(std::min(a + pbits, end_bits));
    }
    std::vector<uint64_t> cand(lo.size());
    {
        DevBuf<uint64_t> dlo, dhi, dc;
        HIPCHK(dlo.alloc(lo.size()));
        HIPCHK(dhi.alloc(lo.size()));
        HIPCHK(dc.alloc(lo.size()));
        if (!lo.empty()) {
            HIPCHK(hipMemcpyAsync(dlo.p, lo.data(), 8 * lo.size(), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(dhi.p, hi.data(), 8 * lo.size(), hipMemcpyHostToDevice, s));
            HIPCHK(ppg_launch_block_find(s, B.comp, B.nwords, dlo.p, dhi.p, dc.p, (int)lo.size(), 1));
            HIPCHK(hipMemcpyAsync(cand.data(), dc.p, 8 * lo.size(), hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipStreamSynchronize(s));
    }
    if (const char *e = getenv("PPG_IX_PERTURB")) {
        // test hook: every n-th candidate moved one bit off its block start -- a false start the
        // chain walk must redo from the real block end (tests/test_index_gpu.py)
        const long n = atol(e);
        for (size_t i = 0; n > 0 && i < cand.size(); i++)
            if (i % (size_t)n == (size_t)n - 1 && cand[i] != ~0ull && cand[i] + 1 < end_bits) cand[i] += 1;
    }
    if (getenv("PPG_IX_PERTURB_LAST")) {
        // test hook: the LAST candidate moved one bit back, into the previous block --
        // the member's last piece then starts inside its predecessor's last block, and next_piece
        // must redo it from that block's end (tests/test_index_gpu.py)
        for (size_t i = cand.size(); i-- > 0;)
            if (cand[i] != ~0ull) {
                if (cand[i] > d0 + 1) cand[i] -= 1;
                break;
            }
    }
    std::vector<Piece> pieces{{0, d0}};
    for (uint64_t c : cand)
        if (c != ~0ull) pieces.push_back({(uint32_t)pieces.size(), c});
    const uint32_t m = (uint32_t)pieces.size();
    stat[0] = ms_since(t);

    // ---- 2. pass 1: block ends + speculative tails ----
    t = Clock::now();
    // slots [0, m): the pieces; [m, m + nspare): speculative redos (below)
    const uint32_t nspare = spare_slots();
    const uint32_t nslots = m + nspare;
    B.nslots = nslots;
    B.hjobs.resize(nslots);
    B.hres.assign(nslots, PpgInflateResult{});
    B.own_blocks.assign(nslots, {});
    uint64_t nblk_total = 0;
    uint32_t max_cap = 0;
    for (uint32_t q = 0; q < m; q++) {
        const uint64_t stop = q + 1 < m ? pieces[q + 1].start : ~0ull;
        const uint64_t span = (q + 1 < m ? stop : end_bits) - pieces[q].start;
        PpgInflateJob &J = B.hjobs[q];
        J = PpgInflateJob{};
        J.bit_start = pieces[q].start;
        J.bit_limit = 8ull * (uint64_t)len;
        J.out_off = (uint64_t)q * kRing;
        J.dict_off = 0;
        J.expect_end = ~0ull;
        J.stop_bit = stop;
        J.blk_off = (uint32_t)nblk_total;
        if (span >= (1ull << 31)) return PPG_UNSUPPORTED;   // the decoder's piece-relative bit positions are 32-bit
        J.blk_cap = (uint32_t)std::min<uint64_t>(span / 8 / 2048 + 64, 1u << 24);
        max_cap = std::max(max_cap, J.blk_cap);
        nblk_total += J.blk_cap;
    }
    const uint32_t spare_cap = std::min<uint32_t>(2 * max_cap, 1u << 24);
    const uint64_t spare_blk = nblk_total;
    nblk_total += (uint64_t)nspare * spare_cap;
    if (nblk_total >= (1ull << 31)) return PPG_UNSUPPORTED;
    B.hblk.reserve((size_t)(len / 20000) + 4096);   // ~one dynamic block per 30 KB of gzip, grown if more
    B.hpos.assign(nslots, 0);
    HIPCHK(B.blk.alloc(nblk_total));
    HIPCHK(B.ring.alloc((size_t)nslots * 2 * kRing));
    HIPCHK(B.ta.alloc((size_t)nslots * 2 * kWin));
    {
        std::vector<uint16_t> ident(kWin);
        for (int i = 0; i < kWin; i++) ident[i] = (uint16_t)i;
        HIPCHK(B.ident.alloc(2 * kWin));
        HIPCHK(hipMemcpy(B.ident.p, ident.data(), 2 * kWin, hipMemcpyHostToDevice));
    }
    if (getenv("PPG_IX_VERBOSE")) fprintf(stderr, "[ix] pass 1 setup %.1f ms\n", ms_since(t));
    {
        std::vector<uint32_t> all(m);
        for (uint32_t q = 0; q < m; q++) all[q] = q;
        int rc = B.run_pass1(all, false);
        if (rc) return rc;
    }
    stat[1] = ms_since(t);

    // walk the pieces in order: a piece is real iff its predecessor (real) ended at its start
    t = Clock::now();
    int redo1 = 0;
    // the first piece after piece j's last block end E: pieces starting inside that block are false
    // starts and are dropped, except the last one before E's successor -- or the member's last
    // piece, when no piece starts at or past E (the finder never offers the final block, whose
    // start is not an inner one) -- which is redone from E
    auto next_piece = [&](size_t j, uint64_t E) {
        size_t k = j + 1;
        while (k + 1 < pieces.size() && pieces[k].start < E && pieces[k + 1].start <= E) k++;
        return k;
    };
    // Speculative redos, one launch: every piece k whose predecessor j (if real) ends somewhere
    // else than k starts is decoded again from that end, into a spare slot.  The walk below takes a
    // spare when it reaches k from the same end; a wrong guess (j itself a false start) is never
    // reached, and a false start beyond the spares is redone serially there.
    std::vector<std::pair<uint64_t, uint32_t>> spec(m, {~0ull, 0});   // piece k -> (E, spare slot)
    {
        std::vector<uint32_t> spares;
        for (size_t j = 0; j + 1 < m && spares.size() < nspare; j++) {
            const PpgInflateResult &r = B.hres[j];
            if (r.status != PPG_OK || r.nblocks == 0 || r.last || (r.flags & PPG_FLAG_BLK_FULL)) continue;
            uint32_t nb = 0;
            const uint64_t E = B.blocks((uint32_t)j, nb)[nb - 1].end_bit;
            const size_t k = next_piece(j, E);
            if (k >= m || pieces[k].start == E || spec[k].first != ~0ull) continue;
            const uint32_t q = m + (uint32_t)spares.size();
            PpgInflateJob J = B.hjobs[pieces[k].slot];
            J.bit_start = E;
            if (J.stop_bit != ~0ull && J.stop_bit <= E) J.stop_bit = E + 1;
            const uint64_t span = (J.stop_bit != ~0ull ? J.stop_bit : end_bits) - E;
            if (span >= (1ull << 31)) continue;
            J.out_off = (uint64_t)q * kRing;
            J.blk_off = (uint32_t)(spare_blk + (uint64_t)(q - m) * spare_cap);
            J.blk_cap = spare_cap;
            B.hjobs[q] = J;
            spec[k] = {E, q};
            spares.push_back(q);
        }
        int rc = B.run_pass1(spares, false);
        if (rc) return rc;
        stat[16] = (double)spares.size();
    }
    std::vector<Piece> real;
    {
        size_t j = 0;
        for (;;) {
            const uint32_t q = pieces[j].slot;
            PpgInflateResult &r = B.hres[q];
            if (r.status == PPG_OK && (r.flags & PPG_FLAG_BLK_FULL)) {
                // more blocks than the slot holds: decode this piece alone into a big list
                PpgInflateJob &J = B.hjobs[q];
                const uint64_t span = (J.stop_bit != ~0ull ? J.stop_bit : end_bits) - J.bit_start;
                J.blk_off = 0;
                J.blk_cap = (uint32_t)std::min<uint64_t>(span / 10 + 64, 1u << 30);
                HIPCHK(B.bigblk.alloc((size_t)J.blk_cap));
                int rc = B.run_pass1({q}, true);
                if (rc) return rc;
                B.own_blocks[q] = B.hblk_big;
                redo1++;
                continue;
            }
            if (r.status != PPG_OK || r.nblocks == 0) return r.status != PPG_OK ? r.status : PPG_DATA_ERROR;
            real.push_back(pieces[j]);
            if (r.last) break;
            uint32_t nb = 0;
            const PpgBlockEnd *bl = B.blocks(q, nb);
            const uint64_t E = bl[nb - 1].end_bit;
            const size_t k = next_piece(j, E);
            if (k >= pieces.size()) return PPG_DATA_ERROR;   // a non-final piece must be followed by one
            if (pieces[k].start != E) {
                redo1++;
                if (spec[k].first == E) {
                    pieces[k] = Piece{spec[k].second, E};       // decoded from E already
                } else {
                    // false start: decode piece k again from the real block end
                    pieces[k].start = E;
                    PpgInflateJob &J = B.hjobs[pieces[k].slot];
                    J.bit_start = E;
                    B.own_blocks[pieces[k].slot].clear();
                    if (J.stop_bit != ~0ull && J.stop_bit <= E) J.stop_bit = E + 1;
                    int rc = B.run_pass1({pieces[k].slot}, false);
                    if (rc) return rc;
                    stat[17] += 1;                              // serial redos (no spare)
                }
            }
            j = k;
        }
    }
    stat[2] = ms_since(t);

    // ---- 3. exact starting histories from the symbolic tails ----
    t = Clock::now();
    const size_t np = real.size();
    DevBuf<uint8_t> W;                  // W[j]: history of real piece j; W[np]: the member's last 32 KiB
    HIPCHK(W.alloc((np + 1) * kWin));
    HIPCHK(hipMemsetAsync(W.p, 0, kWin, s));
    {
        std::vector<uint32_t> sl(np);
        for (size_t j = 0; j < np; j++) sl[j] = real[j].slot;
        DevBuf<uint32_t> dsl;
        DevBuf<uint16_t> maps;          // composed per-group maps
        HIPCHK(dsl.alloc(np));
        HIPCHK(maps.alloc((size_t)ppg_resolve_groups((int)np) * kWin));
        HIPCHK(hipMemcpyAsync(dsl.p, sl.data(), 4 * np, hipMemcpyHostToDevice, s));
        HIPCHK(ppg_launch_resolve(s, B.ta.p, nullptr, dsl.p, (int)np, W.p, maps.p));
        HIPCHK(hipStreamSynchronize(s));
    }
    // pass 1's device state is spent (block lists live on the host): ~190 KiB per slot
    for (DevBuf<uint8_t> *b : {&B.ring, &B.ta, &B.ident}) b->release();
    B.blk.release();
    B.bigblk.release();
    B.dense.release();
    stat[9] = ms_since(t);

    // ---- 4. pass 2: exact output, batch by batch ----
    t = Clock::now();
    std::vector<uint64_t> U(np), O(np + 1, 0);
    size_t max_u = 0;
    for (size_t j = 0; j < np; j++) {
        U[j] = B.hres[real[j].slot].produced;
        O[j + 1] = O[j] + U[j];
        max_u = std::max<size_t>(max_u, U[j]);
        if (U[j] >= (1ull << 31)) return PPG_UNSUPPORTED;
    }
    const uint64_t total = O[np];
    uint64_t cap = out_capacity > 0 ? (uint64_t)out_capacity : 0;
    if (!cap) {
        size_t fr = 0, tot = 0;
        HIPCHK(hipMemGetInfo(&fr, &tot));
        const uint64_t avail = fr > (4ull << 30) ? (uint64_t)fr - (4ull << 30) : (uint64_t)fr / 2;
        // 96 GiB by default: a 204 GB buffer (the whole 50 GB member) cost 2.07 s of hipMalloc when
        // the previous call's had just been freed; two 96 GiB batches decode in 5.47 s both times
        // (bench.py --create-index --ix-capacity-gib, r02)
        cap = std::min<uint64_t>(std::min<uint64_t>(total, avail), kPass2Cap);
    }
    cap = std::max<uint64_t>(cap, max_u);
    DevBuf<uint8_t> out;
    HIPCHK(out.alloc((size_t)cap + 64));
    HIPCHK(hipMemsetAsync(out.p + cap, 0, 64, s));
    stat[15] = ms_since(t);   // the pass-2 output buffer's allocation
    DevBuf<PpgInflateJob> jobs2;
    DevBuf<PpgInflateResult> res2;
    DevBuf<uint8_t> tmp;                // pass-2 tails of a batch (checked against W)
    DevBuf<PpgSpan> spans;
    DevBuf<PpgAtStats> dstats;
    DevBuf<uint8_t> dwin;
    HIPCHK(jobs2.alloc(np));
    HIPCHK(res2.alloc(np));

    // Core.cs:79-110 state carried across batches
    const int64_t threshold = (int64_t)(uint32_t)(chunksize - 8u);
    int64_t records = 0, last_at = -1, last_mark = 0;   // last_mark: output of the last Point or side point
    int batches = 0;
    uint64_t nblocks_seen = 0;
    static const bool verbose = getenv("PPG_IX_VERBOSE") != nullptr;
    struct Ev { hipEvent_t e[6] = {}; ~Ev() { for (auto x : e) if (x) (void)hipEventDestroy(x); } } vevs;
    hipEvent_t *vev = vevs.e;
    if (verbose)
        for (int i = 0; i < 6; i++) HIPCHK(hipEventCreate(&vev[i]));
    // CRC-32 of the output (RFC 1952 trailer), raw register R(0, output so far) folded per batch
    static const CrcTables crc_tabs;
    DevBuf<uint32_t> crc_dtab, crc_seg;
    HIPCHK(crc_dtab.alloc(2048));
    HIPCHK(hipMemcpyAsync(crc_dtab.p, crc_tabs.dev, sizeof crc_tabs.dev, hipMemcpyHostToDevice, s));
    uint32_t crc_raw = 0;
    double t_census = 0;
    ix = ppg_index{};
    std::vector<uint8_t> zeros(kWin, 0);
    ix.add_point(0, hl, 0, 0, zeros.data(), nullptr, 0);   // right after the gzip header (Core.cs:101-102)
    // The Points' windows land in ix.windows: reserve it for the Point count estimated from the '@'
    // density of a sample of the resolved histories, and fault its pages in on host threads while
    // the first batch decodes (r03: ~30 ms per 860 MB of windows when done in line).  A low
    // estimate only means grow() reallocates later, as without it.
    struct Joiner {
        std::vector<std::thread> t;
        void join() { for (auto &x : t) x.join(); t.clear(); }
        ~Joiner() { join(); }
    } prefaulting;
    {
        const size_t ns = std::min<size_t>(np, 64);
        std::vector<uint8_t> smp(ns * kWin);
        for (size_t i = 0; i < ns; i++)
            HIPCHK(hipMemcpyAsync(smp.data() + i * kWin, W.p + (1 + i * np / ns) * kWin, kWin, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const size_t ats = (size_t)std::count(smp.begin(), smp.end(), (uint8_t)'@');
        if (ats && threshold > 0) {
            const double per_point = (double)threshold * (double)smp.size() / (double)ats;   // output bytes
            const size_t est = std::min<size_t>((size_t)(1.1 * (double)total / per_point) + 64, total / kWin + 64);
            ix.windows.reserve(ix.windows.size() + est * kWin);
            uint8_t *a = ix.windows.data() + ix.windows.size();
            const size_t n = ix.windows.capacity() - ix.windows.size(), part = (n / 8 + 4095) & ~(size_t)4095;
            for (int q = 0; q < 8; q++) {
                const size_t lo = std::min(n, q * part), hi = std::min(n, lo + part);
                if (hi > lo) prefaulting.t.emplace_back([=] { prefault(a + lo, hi - lo); });
            }
        }
    }

    std::vector<PpgInflateJob> h2(np);
    for (size_t j = 0; j < np; j++) {
        PpgInflateJob &J = h2[j];
        J = PpgInflateJob{};
        J.bit_start = real[j].start;
        J.bit_limit = 8ull * (uint64_t)len;
        J.out_len = U[j];
        J.dict_off = (uint64_t)j * kWin;
        J.expect_end = ~0ull;
    }
    // a second stream for a batch's '@' census (stats kernel), a third for its tails check and CRC,
    // which follow the census and overlap the host's walk and window copies (r03: census 45 ms +
    // CRC 49 ms per 100 GB batch, one after the other, before the walk could start)
    // (declared before the streams: their destructor drains the copies into it)
    struct Pending {
        bool on = false;
        size_t b0 = 0, nbat = 0;
        uint64_t nb_out = 0;
        std::vector<uint32_t> hseg, hd;
    } pend;
    struct StreamEv {
        hipStream_t s = nullptr, s3 = nullptr;
        hipEvent_t e = nullptr, e2 = nullptr;
        ~StreamEv() {
            // an early return can leave copies in flight
            for (hipStream_t x : {s, s3}) if (x) (void)hipStreamSynchronize(x);
            for (hipEvent_t x : {e, e2}) if (x) (void)hipEventDestroy(x);
            for (hipStream_t x : {s, s3}) if (x) (void)hipStreamDestroy(x);
        }
    } side;
    HIPCHK(hipStreamCreateWithFlags(&side.s, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&side.e, hipEventDisableTiming));
    const hipStream_t s2 = side.s;
    HIPCHK(hipStreamCreateWithFlags(&side.s3, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&side.e2, hipEventDisableTiming));
    const hipStream_t s3 = side.s3;
    DevBuf<PpgGather> gat_tails;
    // a batch's deferred checks, folded in before the next batch overwrites the output
    auto settle = [&]() -> int {
        if (!pend.on) return PPG_OK;
        if (!pend.hseg.empty())
            HIPCHK(hipMemcpyAsync(pend.hseg.data(), crc_seg.p, 4 * pend.hseg.size(), hipMemcpyDeviceToHost, s3));
        HIPCHK(hipMemcpyAsync(pend.hd.data(), B.diff.p, 4 * pend.nbat, hipMemcpyDeviceToHost, s3));
        HIPCHK(hipStreamSynchronize(s3));
        pend.on = false;
        if (verbose) {
            float b = 0;
            HIPCHK(hipEventElapsedTime(&b, vev[2], vev[3]));
            fprintf(stderr, "[ix] pass 2 batch: crc %.1f ms (third stream)\n", b);
        }
        uint32_t r = 0;   // R(0, batch output) = fold of the segments with Z(., kCrcSeg)
        for (uint32_t v : pend.hseg) r = crc_tabs.zseg(r) ^ v;
        crc_raw = (uint32_t)crc32_combine(crc_raw, r, (z_off_t)pend.nb_out);
        for (size_t i = 0; i < pend.nbat; i++)
            if (pend.hd[i]) {
                fprintf(stderr, "ppgpu: GPU CreateIndex: piece %zu does not reproduce its resolved history\n", pend.b0 + i);
                return PPG_DEVICE_ERROR;
            }
        return PPG_OK;
    };
    size_t b0 = 0;
    while (b0 < np) {
        if (int rc = settle()) return rc;
        size_t b1 = b0 + 1;
        while (b1 < np && O[b1 + 1] - O[b0] <= cap) b1++;
        const size_t nbat = b1 - b0;
        batches++;
        for (size_t j = b0; j < b1; j++) h2[j].out_off = O[j] - O[b0];
        // the batch's blocks as output spans (pass 1's block lists), uploaded ahead of the decode
        std::vector<PpgSpan> hs;
        struct BlockRef { uint32_t j; uint64_t end_bit, rel_end; };
        std::vector<BlockRef> refs;
        for (size_t j = b0; j < b1; j++) {
            uint32_t nb = 0;
            const PpgBlockEnd *bl = B.blocks(real[j].slot, nb);
            uint64_t prev = 0;
            for (uint32_t b = 0; b < nb; b++) {
                hs.push_back(PpgSpan{h2[j].out_off + prev, h2[j].out_off + bl[b].out_end});
                refs.push_back(BlockRef{(uint32_t)j, bl[b].end_bit, bl[b].out_end});
                prev = bl[b].out_end;
            }
        }
        std::vector<PpgAtStats> st(hs.size());
        if (!hs.empty()) {
            HIPCHK(spans.alloc(hs.size()));
            HIPCHK(dstats.alloc(hs.size()));
            HIPCHK(hipMemcpyAsync(spans.p, hs.data(), sizeof(PpgSpan) * hs.size(), hipMemcpyHostToDevice, s));
        }
        HIPCHK(hipMemcpyAsync(jobs2.p + b0, h2.data() + b0, sizeof(PpgInflateJob) * nbat, hipMemcpyHostToDevice, s));
        if (verbose) HIPCHK(hipEventRecord(vev[0], s));
        HIPCHK(ppg_launch_inflate(s, ctx->ring_bits, ctx->lit_bits, B.comp, B.nwords, jobs2.p + b0, W.p, out.p,
                                  res2.p + b0, (int)nbat, nullptr));
        if (verbose) HIPCHK(hipEventRecord(vev[1], s));
        HIPCHK(hipEventRecord(side.e, s));
        const auto tb = Clock::now();
        if (!hs.empty()) {   // ---- 4. '@' census of the batch's blocks (second stream) ----
            HIPCHK(hipStreamWaitEvent(s2, side.e, 0));
            if (verbose) HIPCHK(hipEventRecord(vev[4], s2));
            HIPCHK(ppg_launch_at_stats(s2, out.p, spans.p, dstats.p, (int)hs.size()));
            if (verbose) HIPCHK(hipEventRecord(vev[5], s2));
            HIPCHK(hipMemcpyAsync(st.data(), dstats.p, sizeof(PpgAtStats) * hs.size(), hipMemcpyDeviceToHost, s2));
            HIPCHK(hipEventRecord(side.e2, s2));
        }
        // third stream, checked later (settle): every piece must hand on exactly the history the
        // next one was resolved to start with, and the CRC-32 of the batch's output (front-padded
        // to whole kCrcSeg segments, one wave each) -- they overlap the host's walk and windows
        {
            std::vector<PpgGather> g(nbat);
            for (size_t j = b0; j < b1; j++)
                g[j - b0] = PpgGather{h2[j].out_off, (uint64_t)j * kWin, U[j], ~0ull, (uint64_t)(j + 1) * kWin};
            HIPCHK(tmp.alloc(nbat * kWin));
            HIPCHK(B.diff.alloc(nbat));
            HIPCHK(gat_tails.alloc(nbat));
            HIPCHK(hipMemcpyAsync(gat_tails.p, g.data(), sizeof(PpgGather) * nbat, hipMemcpyHostToDevice, s3));
            // after the census, which the host's walk waits for; these overlap that walk
            HIPCHK(hipStreamWaitEvent(s3, hs.empty() ? side.e : side.e2, 0));
            HIPCHK(ppg_launch_gather(s3, out.p, W.p, gat_tails.p, tmp.p, W.p, B.diff.p, (int)nbat));
            pend.nb_out = O[b1] - O[b0];
            const uint64_t crc_pad = (kCrcSeg - pend.nb_out % kCrcSeg) % kCrcSeg;
            const uint64_t nseg = (pend.nb_out + crc_pad) / kCrcSeg;
            HIPCHK(crc_seg.alloc(std::max<uint64_t>(nseg, 1)));
            if (verbose) HIPCHK(hipEventRecord(vev[2], s3));
            HIPCHK(ppg_launch_crc(s3, out.p, pend.nb_out, crc_pad, crc_dtab.p, crc_seg.p, nseg));
            if (verbose) HIPCHK(hipEventRecord(vev[3], s3));
            // (read back in settle: a copy into pageable memory holds the host until it has run)
            pend.hseg.assign(nseg, 0);
            pend.hd.assign(nbat, 0);
            pend.b0 = b0;
            pend.nbat = nbat;
            pend.on = true;
        }
        std::vector<PpgInflateResult> r2(nbat);
        HIPCHK(hipMemcpyAsync(r2.data(), res2.p + b0, sizeof(PpgInflateResult) * nbat, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipStreamSynchronize(s2));   // (before any return: its copy lands in st)
        for (size_t i = 0; i < nbat; i++) {
            if (r2[i].status != PPG_OK) return r2[i].status;
            if (r2[i].produced != U[b0 + i]) return PPG_DATA_ERROR;
        }
        if (verbose) {
            float a = 0, c = 0, d = 0;
            HIPCHK(hipEventElapsedTime(&a, vev[0], vev[1]));
            HIPCHK(hipEventElapsedTime(&c, vev[4], vev[5]));
            HIPCHK(hipEventElapsedTime(&d, vev[1], vev[5]));
            fprintf(stderr, "[ix] pass 2 batch %d: inflate %.1f ms, census kernel %.1f (ends %.1f after the inflate); "
                            "census on the host %.1f ms after launch\n", batches, a, c, d, ms_since(tb));
        }

        // ---- 4. the Points among the batch's blocks (Core.cs:79-110) ----
        const auto tc = Clock::now();
        const double t_stats = 0;   // (the census ran on the second stream, beside the CRC)
        const bool final_batch = b1 == np;
        struct Pick { int64_t bits, input, output; uint32_t j; uint64_t rel; int64_t off_len; };
        std::vector<Pick> picks;
        struct Side { uint64_t end_bit; int64_t output; uint32_t j; uint64_t rel; };
        std::vector<Side> sides;
        for (size_t i = 0; i < refs.size(); i++) {
            const BlockRef &br = refs[i];
            const uint64_t gs = O[br.j] + (hs[i].lo - h2[br.j].out_off);
            const uint64_t ge = O[br.j] + br.rel_end;
            const PpgAtStats &a = st[i];
            if (a.count) {                                  // SURVEY Q4 (Core.cs:93)
                const int64_t first = (int64_t)gs + a.first;
                if (last_at < 0 ? first > kMaxRun : first - last_at > kMaxRun) return PPG_INDEX_OUT_OF_RANGE;
                if ((int64_t)a.max_gap > kMaxRun) return PPG_INDEX_OUT_OF_RANGE;
                last_at = (int64_t)gs + a.last;
                records += a.count;
            }
            if (final_batch && i + 1 == refs.size()) break;  // the final block: no Point (data_type & 64)
            const int64_t input = (int64_t)((br.end_bit + 7) >> 3), bits = input * 8 - (int64_t)br.end_bit;
            if (ge == 0) {
                picks.push_back(Pick{bits, input, 0, br.j, 0, -1});
            } else if (records > threshold) {
                const int64_t off_len = (int64_t)ge - (last_at < 0 ? 0 : last_at);
                if (off_len > kMaxRun) return PPG_INDEX_OUT_OF_RANGE;
                picks.push_back(Pick{bits, input, (int64_t)ge, br.j, br.rel_end, off_len});
                records = 0;
                last_mark = (int64_t)ge;
                // a side point at this output (an empty block before this one) would not be inside a chunk
                if (!sides.empty() && sides.back().output == (int64_t)ge) sides.pop_back();
                if (sides.empty() && !ix.side_out.empty() && ix.side_out.back() == (int64_t)ge) {
                    ix.side_bit.pop_back();
                    ix.side_out.pop_back();
                    ix.side_win.resize(ix.side_win.size() - kWin);
                }
            } else if (side_bytes > 0 && (int64_t)ge - last_mark >= side_bytes &&
                       (sides.empty() || sides.back().output != (int64_t)ge)) {
                // a side point: a block start inside the current chunk, side_bytes past the last mark
                sides.push_back(Side{br.end_bit, (int64_t)ge, br.j, br.rel_end});
                last_mark = (int64_t)ge;
            }
        }
        nblocks_seen += refs.size();
        const double t_walk = ms_since(tc);
        // windows of the picked Points, then the side points', gathered on the device in index order
        // and copied straight onto the index's window arrays (a zero-output Point reads W[0]: zeros)
        std::vector<PpgGather> gw;
        for (const Pick &p : picks)
            gw.push_back(p.output > 0 ? PpgGather{h2[p.j].out_off, (uint64_t)p.j * kWin, p.rel, ~0ull, 0}
                                      : PpgGather{0, 0, 0, ~0ull, 0});
        for (const Side &d : sides) gw.push_back(PpgGather{h2[d.j].out_off, (uint64_t)d.j * kWin, d.rel, ~0ull, 0});
        // grown to the whole member's projected size (at least x1.5): an exact per-batch reserve
        // recopied every window so far on every batch (quadratic in the batch count)
        const double proj = 1.02 * (double)total / (double)std::max<uint64_t>(O[b1], 1);
        prefaulting.join();   // (before grow() may move the array)
        grow(ix.pts, ix.pts.size() + picks.size(), proj);
        grow(ix.windows, ix.windows.size() + picks.size() * kWin, proj);
        grow(ix.side_bit, ix.side_bit.size() + sides.size(), proj);
        grow(ix.side_out, ix.side_out.size() + sides.size(), proj);
        grow(ix.side_win, ix.side_win.size() + sides.size() * kWin, proj);
        const size_t w0 = ix.windows.size(), s0 = ix.side_win.size();
        ix.windows.resize(w0 + picks.size() * kWin);          // uninitialised (ByteVec)
        ix.side_win.resize(s0 + sides.size() * kWin);
        const auto tw = Clock::now();
        {   // fault the new window pages in from 8 threads (huge pages where allowed)
            std::thread th[8];
            const size_t nw = picks.size() * kWin, part = (nw / 8 + 4095) & ~(size_t)4095;
            for (int q = 0; q < 8; q++) {
                const size_t a = std::min(nw, q * part), z = std::min(nw, a + part);
                th[q] = std::thread([&, a, z] { if (z > a) prefault(ix.windows.data() + w0 + a, z - a); });
            }
            for (auto &x : th) x.join();
        }
        const double t_fault = ms_since(tw);
        double t_alloc = 0, t_gat = 0;
        if (!gw.empty()) {
            HIPCHK(B.gat.alloc(gw.size()));
            HIPCHK(dwin.alloc(gw.size() * kWin));
            t_alloc = ms_since(tw) - t_fault;
            HIPCHK(hipMemcpyAsync(B.gat.p, gw.data(), sizeof(PpgGather) * gw.size(), hipMemcpyHostToDevice, s));
            HIPCHK(ppg_launch_gather(s, out.p, W.p, B.gat.p, dwin.p, nullptr, nullptr, (int)gw.size()));
            if (verbose) {
                HIPCHK(hipStreamSynchronize(s));
                t_gat = ms_since(tw) - t_fault - t_alloc;
            }
            if (int rc = copy_d2h_staged(ctx, s, ix.windows.data() + w0, dwin.p, picks.size() * kWin)) return rc;
            if (int rc = copy_d2h_staged(ctx, s, ix.side_win.data() + s0, dwin.p + picks.size() * kWin, sides.size() * kWin))
                return rc;
        }
        for (const Side &d : sides) {
            ix.side_bit.push_back((int64_t)d.end_bit);
            ix.side_out.push_back(d.output);
        }
        for (size_t i = 0; i < picks.size(); i++) {
            const Pick &p = picks[i];
            const uint8_t *w = ix.windows.data() + w0 + i * kWin;
            if (p.output == 0)
                ix.add_point_fields((int)p.bits, p.input, 0, nullptr, 0);
            else
                ix.add_point_fields((int)p.bits, p.input, p.output, w + kWin - p.off_len, (size_t)p.off_len);
        }
        t_census += ms_since(tc);
        if (verbose)
            fprintf(stderr, "[ix] batch %d: %zu pieces, %zu blocks, census: stats %.1f ms, walk %.1f, windows %.1f (%zu; "
                            "grow %.1f, prefault %.1f, alloc %.1f, gather %.1f, copy + points %.1f)\n",
                    batches, nbat, hs.size(), t_stats, t_walk - t_stats, ms_since(tc) - t_walk, gw.size(),
                    std::chrono::duration<double, std::milli>(tw - tc).count() - t_walk, t_fault, t_alloc, t_gat,
                    ms_since(tw) - t_fault - t_alloc - t_gat);
        b0 = b1;
    }
    if (int rc = settle()) return rc;
    stat[3] = ms_since(t) - t_census;
    stat[4] = t_census;
    stat[10] = (double)batches;

    // ---- end of the member: trailer (RFC 1952: CRC32, ISIZE) and the final Point (Core.cs:123) ----
    uint32_t nb = 0;
    const PpgBlockEnd *bl = B.blocks(real.back().slot, nb);
    const int64_t tpos = (int64_t)((bl[nb - 1].end_bit + 7) >> 3);
    if (tpos + 8 > len) return PPG_DATA_ERROR;
    if (tpos + 8 < len) return PPG_UNSUPPORTED;       // another member or trailing bytes
    const uint32_t isize = (uint32_t)trailer[4] | ((uint32_t)trailer[5] << 8) | ((uint32_t)trailer[6] << 16) |
                           ((uint32_t)trailer[7] << 24);
    if (isize != (uint32_t)total) return PPG_DATA_ERROR;                   // zlib: "incorrect length check"
    {
        const uint32_t want = (uint32_t)trailer[0] | ((uint32_t)trailer[1] << 8) | ((uint32_t)trailer[2] << 16) |
                              ((uint32_t)trailer[3] << 24);
        // crc32(output) = R(~0, output) ^ ~0 = R(0, output) ^ Z(~0, |output|) ^ ~0
        const uint32_t got = crc_raw ^ (uint32_t)crc32_combine(0xFFFFFFFFu, 0, (z_off_t)total) ^ 0xFFFFFFFFu;
        if (got != want) return PPG_DATA_ERROR;                                 // zlib: "incorrect data check"
    }
    if (last_at < 0 ? (int64_t)total > kMaxRun : (int64_t)total - 1 - last_at >= kMaxRun) return PPG_INDEX_OUT_OF_RANGE;
    {
        std::vector<uint8_t> w(kWin);
        HIPCHK(hipMemcpy(w.data(), W.p + np * kWin, kWin, hipMemcpyDeviceToHost));
        ix.add_point(0, len, (int64_t)total, 0, w.data(), nullptr, 0);
    }
    stat[5] = ms_since(t_all);
    stat[6] = (double)m;
    stat[7] = (double)np;
    stat[8] = (double)redo1;
    stat[11] = (double)nblocks_seen;
    stat[12] = (double)ix.pts.size();
    stat[13] = (double)total;
    return PPG_OK;
}

extern "C" {

int ppg_index_build_gpu_side(ppg_ctx *ctx, const void *gz, int64_t gz_len, int gz_on_device, uint32_t chunksize,
                             int64_t piece_bytes, int64_t out_capacity, int64_t side_bytes, ppg_index **out);

int ppg_index_build_gpu(ppg_ctx *ctx, const void *gz, int64_t gz_len, int gz_on_device, uint32_t chunksize,
                        int64_t piece_bytes, int64_t out_capacity, ppg_index **out) {
    return ppg_index_build_gpu_side(ctx, gz, gz_len, gz_on_device, chunksize, piece_bytes, out_capacity, 0, out);
}

int ppg_index_side_count(const ppg_index *ix) { return ix ? (int)ix->side_out.size() : -1; }

int ppg_index_side_points(const ppg_index *ix, int64_t *bit, int64_t *output, uint8_t *windows) {
    if (!ix) return PPG_ARG_ERROR;
    const size_t n = ix->side_out.size();
    if (bit) std::copy(ix->side_bit.begin(), ix->side_bit.end(), bit);
    if (output) std::copy(ix->side_out.begin(), ix->side_out.end(), output);
    if (windows && n) memcpy(windows, ix->side_win.data(), n * kWin);
    return PPG_OK;
}

int ppg_index_set_side_points(ppg_index *ix, int32_t n, const int64_t *bit, const int64_t *output,
                              const uint8_t *windows) {
    if (!ix || n < 0 || (n && (!bit || !output || !windows))) return PPG_ARG_ERROR;
    for (int32_t i = 1; i < n; i++)
        if (output[i] <= output[i - 1] || bit[i] <= bit[i - 1]) return PPG_ARG_ERROR;
    // each point strictly inside one chunk of the index, in output AND in compressed bits (ADVICE
    // r04: a point outside its chunk's bit range failed every request of a shared Decompress launch)
    const auto &P = ix->pts;
    if (n && P.size() < 2) return PPG_ARG_ERROR;
    for (int32_t i = 0, c = 0; i < n; i++) {
        while ((size_t)c + 1 < P.size() && output[i] >= P[(size_t)c + 1].output) c++;
        if ((size_t)c + 1 >= P.size() || output[i] <= P[(size_t)c].output) return PPG_ARG_ERROR;
        const int64_t b0 = 8 * P[(size_t)c].input - P[(size_t)c].bits, b1 = 8 * P[(size_t)c + 1].input - P[(size_t)c + 1].bits;
        if (bit[i] <= b0 || bit[i] >= b1) return PPG_ARG_ERROR;
    }
    ix->side_bit.assign(bit, bit + n);
    ix->side_out.assign(output, output + n);
    ix->side_win.resize((size_t)n * kWin);
    if (n) memcpy(ix->side_win.data(), windows, (size_t)n * kWin);
    return PPG_OK;
}

int ppg_index_build_gpu_side(ppg_ctx *ctx, const void *gz, int64_t gz_len, int gz_on_device, uint32_t chunksize,
                             int64_t piece_bytes, int64_t out_capacity, int64_t side_bytes, ppg_index **out) {
    if (!ctx || !gz || gz_len <= 0 || !out) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t hn = std::min<int64_t>(gz_len, 65536);
    std::vector<uint8_t> head((size_t)hn);
    uint8_t trailer[8] = {0};
    DevBuf<uint8_t> own;
    const uint8_t *d = (const uint8_t *)gz;
    if (gz_on_device) {
        if (((uintptr_t)gz & 3) != 0) return PPG_ARG_ERROR;
        HIPCHK(hipMemcpy(head.data(), gz, (size_t)hn, hipMemcpyDeviceToHost));
        if (gz_len >= 8) HIPCHK(hipMemcpy(trailer, d + gz_len - 8, 8, hipMemcpyDeviceToHost));
    } else {
        memcpy(head.data(), gz, (size_t)hn);
        if (gz_len >= 8) memcpy(trailer, d + gz_len - 8, 8);
        HIPCHK(own.alloc((size_t)gz_len + 64));
        HIPCHK(hipMemsetAsync(own.p + gz_len, 0, 64, s));
        HIPCHK(hipMemcpyAsync(own.p, gz, (size_t)gz_len, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        d = own.p;
    }
    auto ix = std::make_unique<ppg_index>();
    const int rc = build_index_gpu(ctx, d, gz_len, head.data(), hn, trailer, chunksize, piece_bytes, out_capacity,
                                   side_bytes, *ix);
    if (rc != PPG_OK) return rc;
    *out = ix.release();
    return PPG_OK;
}

int ppg_index_build_gpu_file(ppg_ctx *ctx, const char *gz_path, uint32_t chunksize, int64_t piece_bytes,
                             ppg_index **out) {
    if (!ctx || !gz_path || !out) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int fd = open(gz_path, O_RDONLY);
    if (fd < 0) return PPG_IO_ERROR;
    struct FdClose { int fd; ~FdClose() { close(fd); } } fdc{fd};
    const int64_t len = (int64_t)lseek(fd, 0, SEEK_END);
    if (len <= 0) return PPG_DATA_ERROR;
    // whole member into HBM: pread into two pinned 64 MiB halves, H2D alternating
    const auto t0 = std::chrono::steady_clock::now();
    DevBuf<uint8_t> dev;
    HIPCHK(dev.alloc((size_t)len + 64));
    HIPCHK(hipMemsetAsync(dev.p + len, 0, 64, s));
    constexpr int64_t kStage = 64 << 20;
    PinnedBuf pin;
    HIPCHK(pin.alloc(2 * kStage));
    hipEvent_t ev[2];
    HIPCHK(hipEventCreate(&ev[0]));
    HIPCHK(hipEventCreate(&ev[1]));
    struct EvFree { hipEvent_t *e; ~EvFree() { (void)hipEventDestroy(e[0]); (void)hipEventDestroy(e[1]); } } evf{ev};
    bool used[2] = {false, false};
    int64_t done = 0;
    for (int h = 0; done < len; h ^= 1) {
        if (used[h]) HIPCHK(hipEventSynchronize(ev[h]));
        const int64_t n = std::min(kStage, len - done);
        uint8_t *p = pin.p + h * kStage;
        int64_t got = 0;
        while (got < n) {
            const ssize_t r = pread(fd, p + got, (size_t)(n - got), (off_t)(done + got));
            if (r <= 0) return PPG_IO_ERROR;
            got += r;
        }
        HIPCHK(hipMemcpyAsync(dev.p + done, p, (size_t)n, hipMemcpyHostToDevice, s));
        HIPCHK(hipEventRecord(ev[h], s));
        used[h] = true;
        done += n;
    }
    HIPCHK(hipStreamSynchronize(s));
    const int64_t hn = std::min<int64_t>(len, 65536);
    std::vector<uint8_t> head((size_t)hn);
    uint8_t trailer[8] = {0};
    if (pread(fd, head.data(), (size_t)hn, 0) != (ssize_t)hn) return PPG_IO_ERROR;
    if (len >= 8 && pread(fd, trailer, 8, (off_t)(len - 8)) != 8) return PPG_IO_ERROR;
    auto ix = std::make_unique<ppg_index>();
    const double upload = ms_since(t0);
    const int rc = build_index_gpu(ctx, dev.p, len, head.data(), hn, trailer, chunksize, piece_bytes, 0, 0, *ix);
    ctx->ix_stats[14] = upload;
    if (rc != PPG_OK) return rc;
    *out = ix.release();
    return PPG_OK;
}

int ppg_index_build_gpu_stats(ppg_ctx *ctx, double *vals, int32_t n) {
    if (!ctx || !vals || n < 0) return PPG_ARG_ERROR;
    for (int32_t i = 0; i < n && i < kIxStats; i++) vals[i] = ctx->ix_stats[i];
    return PPG_OK;
}

}  // extern "C"

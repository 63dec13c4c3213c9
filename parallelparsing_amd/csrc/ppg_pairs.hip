// ppg_pairs.hip — paired reads behind the C ABI (BASELINE configs[4]; the reference
// only names the goal, /root/reference/README.md:9, and has no code for it).
//
// R1 and R2 are two files whose record i belong together: "SRR<id>.<spot>.<mate>" identifiers with
// equal spot numbers.  Each file is decoded by its own DecompressAll (ppg_shard_run, per-file
// parity); pair number i is R1's and R2's i-th record once the records the reference parses twice
// are dropped (a Point on a record start re-emits that record; ppg_record_keys marks it
// -2).  ppg_pairs_check verifies the pairing on the device:
//
//   keys      each shard's spot keys: the buffer its runs filled batch by batch (ppg_shard_set_keys)
//             or, for a one-batch shard, ppg_record_keys now;
//   dedup     the duplicates' positions (rare: at most one per chunk) found by ppg_key_dups and
//             sorted on the host; the deduplicated numbering is a map, not a copy: record
//             r(i) = i + #{t : D[t] - t <= i} for the sorted duplicate positions D
//             (ppg_key_compact gathers through it, one search per 2,048 keys unless a duplicate
//             falls inside them);
//   exchange  (N ranks, a ppg_comm) a rank holds contiguous record ranges of both files that do
//             not line up across ranks, so pairs are owned evenly by pair number and every key moves
//             to its owner: a status + count all-gather, then one all-to-all-v per file (RCCL
//             grouped ncclSend / ncclRecv over xGMI, or the host transport's shared memory);
//   compare   ppg_pair_compare counts pairs whose keys differ or are missing (< 0) and finds the
//             first one; the counts of the two files must agree too.
#include "ppg_host.h"
#include <chrono>

namespace {
constexpr int64_t kDupKey = -2;   // ppg_record_keys: a record the reference parses twice (Q1)
constexpr uint32_t kCompactSpan = 2048;
}

extern "C" __global__ __launch_bounds__(256) void ppg_key_dups(const int64_t *__restrict__ keys, uint64_t n,
                                                               uint64_t *__restrict__ pos, uint32_t cap,
                                                               uint32_t *__restrict__ count) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        if (keys[i] == kDupKey) {
            const uint32_t c = atomicAdd(count, 1u);
            if (c < cap) pos[c] = i;
        }
}

// #{t < nd : dp[t] <= i}
__device__ __forceinline__ uint32_t dup_shift(const int64_t *__restrict__ dp, uint32_t nd, int64_t i) {
    uint32_t lo = 0, hi = nd;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (dp[mid] <= i) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// out[i - lo] = keys[r(i)] for deduplicated numbers i in [lo, lo + n)
extern "C" __global__ __launch_bounds__(256) void ppg_key_compact(const int64_t *__restrict__ keys,
                                                                  const int64_t *__restrict__ dp, uint32_t nd,
                                                                  uint64_t lo, uint64_t n, int64_t *__restrict__ out) {
    const uint64_t b0 = lo + (uint64_t)blockIdx.x * kCompactSpan;
    const uint64_t b1 = min(b0 + kCompactSpan, lo + n);
    if (b0 >= b1) return;
    const uint32_t s0 = dup_shift(dp, nd, (int64_t)b0), s1 = dup_shift(dp, nd, (int64_t)(b1 - 1));
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256) {
        const uint32_t s = s0 == s1 ? s0 : dup_shift(dp, nd, (int64_t)i);
        out[i - lo] = keys[i + s];
    }
}

// res[0] += pairs i in [0, n) with a[i] != b[i] or a[i] < 0; res[1] = min such i
extern "C" __global__ __launch_bounds__(256) void ppg_pair_compare(const int64_t *__restrict__ a,
                                                                   const int64_t *__restrict__ b, uint64_t n,
                                                                   unsigned long long *__restrict__ res) {
    unsigned long long cnt = 0, first = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const int64_t x = a[i], y = b[i];
        if (x != y || x < 0) {
            cnt++;
            first = min(first, (unsigned long long)i);
        }
    }
    if (cnt) {
        atomicAdd(&res[0], cnt);
        atomicMin(&res[1], first);
    }
}

// ---- record-aligned pair chunks: records packed back to back (ppg_pairs_emit_*) ----
// A segment is a run of consecutive records of one chunk's raw text (raw = offset_k ++ body_k, the
// CombinedMemory of Parsing.cs:72-117), copied to dst + dst with its descriptors rebased by delta.
struct PpgPackSeg {
    const uint8_t *off;       // raw [0, olen): the Point's offset carry (may be null when olen = 0)
    const uint8_t *body;      // raw [olen, ...): the chunk's output (a 64-B readable tail follows)
    const uint32_t *desc;     // the segment's first record's descriptor (n1, n2, n3, n4)
    uint64_t olen;
    uint64_t a, b;            // raw bytes [a, b): ppg_seg_bounds fills them
    uint64_t dst;             // byte offset in the destination
    uint64_t ddst;            // record offset in the destination's descriptors
    uint32_t nrec, first;     // first: the segment starts at its raw's first byte (a = 0)
    int64_t delta;            // added to every descriptor value: the bytes' offset in their half, - a
};

// a = the segment's first byte (0, or the previous record's n4 + 1), b = its last record's n4 + 1
extern "C" __global__ __launch_bounds__(256) void ppg_seg_bounds(PpgPackSeg *__restrict__ seg, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    PpgPackSeg &s = seg[i];
    s.a = s.first ? 0u : (uint64_t)s.desc[-1] + 1u;
    s.b = s.nrec ? (uint64_t)s.desc[4 * (uint64_t)s.nrec - 1] + 1u : s.a;
}

__device__ __forceinline__ uint32_t seg_raw(const PpgPackSeg &s, uint64_t i) {
    return i < s.olen ? s.off[i] : s.body[i - s.olen];
}

// grid (x: stripes of a segment, y: segments); 16-B destination words inside the body part from
// aligned dword loads (alignbyte), the rest -- the offset carry part, an unaligned head and tail --
// byte by byte (each destination byte belongs to exactly one segment)
extern "C" __global__ __launch_bounds__(256) void ppg_pack_segs(const PpgPackSeg *__restrict__ seg, int n,
                                                                uint8_t *__restrict__ dst, uint32_t *__restrict__ ddesc) {
    for (int y = blockIdx.y; y < n; y += gridDim.y) {
        const PpgPackSeg s = seg[y];
        const uint64_t len = s.b - s.a, d0 = s.dst;
        // bytes: raw [a, b) -> dst [d0, d0 + len); body bytes start at destination bd
        const uint64_t bd = d0 + (s.olen > s.a ? s.olen - s.a : 0);
        const uint64_t w0 = (bd + 15) / 16, w1 = (d0 + len) / 16;
        const uint64_t nw = w1 > w0 ? w1 - w0 : 0;
        const uint64_t per = (nw + gridDim.x - 1) / gridDim.x;
        const uint64_t wa = w0 + min(nw, (uint64_t)blockIdx.x * per), wz = w0 + min(nw, (uint64_t)(blockIdx.x + 1) * per);
        const uint64_t body_a = s.a > s.olen ? s.a - s.olen : 0;   // body byte at destination bd
        for (uint64_t w = wa + threadIdx.x; w < wz; w += 256) {
            const uint8_t *src = s.body + body_a + (16 * w - bd);
            const uint32_t *s32 = (const uint32_t *)((uintptr_t)src & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)((uintptr_t)src & 3);
            const uint32_t x0 = s32[0], x1 = s32[1], x2 = s32[2], x3 = s32[3], x4 = s32[4];
            uint4 v;
            v.x = __builtin_amdgcn_alignbyte(x1, x0, sh);
            v.y = __builtin_amdgcn_alignbyte(x2, x1, sh);
            v.z = __builtin_amdgcn_alignbyte(x3, x2, sh);
            v.w = __builtin_amdgcn_alignbyte(x4, x3, sh);
            *(uint4 *)(dst + 16 * w) = v;
        }
        if (blockIdx.x == 0) {
            const uint64_t head = nw ? 16 * w0 - d0 : len;
            for (uint64_t i = threadIdx.x; i < head; i += 256) dst[d0 + i] = (uint8_t)seg_raw(s, s.a + i);
            if (nw)
                for (uint64_t i = 16 * w1 - d0 + threadIdx.x; i < len; i += 256) dst[d0 + i] = (uint8_t)seg_raw(s, s.a + i);
        }
        // descriptors, rebased (u32 arithmetic: a half stays under 4 GiB -- half_max() refuses longer ones)
        const uint64_t nv = 4 * (uint64_t)s.nrec;
        const uint64_t pv = (nv + gridDim.x - 1) / gridDim.x;
        const uint64_t va = min(nv, (uint64_t)blockIdx.x * pv), vz = min(nv, (uint64_t)(blockIdx.x + 1) * pv);
        for (uint64_t i = va + threadIdx.x; i < vz; i += 256)
            ddesc[4 * s.ddst + i] = (uint32_t)((int64_t)s.desc[i] + s.delta);
    }
}

hipError_t ppg_launch_record_keys(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  const PpgParseInfo *info, const uint64_t *base, const uint32_t *recs, int64_t *keys,
                                  int n);

// a shard's state around a batch run again for emission (rerun_launch / rerun_collect)
struct RerunSave {
    int64_t tot = 0;
    float ti = 0, tp = 0, tt = 0;
    int64_t *keys = nullptr;
};

// ppg_pairs_emit_*: the record-aligned pair chunks (see the ABI comment in include/ppgpu.h)
struct PairEmit {
    bool on = false;
    int64_t K = 0, npc = 0;                 // pair chunk size; pair chunks in all
    int64_t j_lo = 0, j_hi = 0;             // this rank's pair chunks
    int64_t next = 0;                       // the next window's first pair chunk
    int64_t w0 = 0, w1 = 0;                 // the current window
    int64_t window_bytes = 0;               // one rank: bytes per window and file (a budget, >= 1 pair chunk)
    ppg_shard *sh[2] = {nullptr, nullptr};
    ppg_comm *comm = nullptr;
    bool exchanged = false;                 // N ranks: the one window is done
    int32_t batch[2] = {-1, -1};            // one rank: the resident output batch of each shard
    int32_t kvalid[2] = {0, 0};             // chunks [0, kvalid) have their record bases (h_base) set
    std::vector<int64_t> blo[2], bhi[2];    // one rank: each batch's deduplicated record range
    std::vector<uint64_t> offst[2];         // chunk k's offset carry in sh->offs
    std::vector<int64_t> pos[2];            // shard positions of the duplicates (sorted)
    // the current window: per pair chunk j (from w0) and file, byte offset / length, first record / count
    std::vector<int64_t> boff[2], blen[2], roff[2], rcnt[2];
    DevBuf<uint8_t> bytes[2];
    DevBuf<uint32_t> desc[2];
    // one rank: the part of pair chunk `next` carried from an earlier batch
    DevBuf<uint8_t> cbytes[2];
    DevBuf<uint32_t> cdesc[2];
    int64_t clen[2] = {0, 0}, cnrec[2] = {0, 0};
    DevBuf<PpgPackSeg> dseg;
    // N ranks: exchange buffers (bytes as int64 words, descriptors as two int64 per record)
    DevBuf<int64_t> sbuf[2], rbuf[2], sdesc[2], rdesc[2];
    RerunSave save[2];
    // fused (ppg_pairs_emit_run): the shards' own first run, batch by batch as the windows advance
    bool fused = false;
    bool done[2] = {false, false};          // the file's last batch has run (shard finished)
    float run_ms[2] = {0, 0};               // its batches' kernel time, as shard_run sums it
    double t_ms[4] = {0, 0, 0, 0};          // batches (re-)run, packing, exchange, total (ms, cumulative)
    int64_t reruns = 0;
    void release() {
        for (int f = 0; f < 2; f++) {
            bytes[f].release(); desc[f].release(); cbytes[f].release(); cdesc[f].release();
            sbuf[f].release(); rbuf[f].release(); sdesc[f].release(); rdesc[f].release();
        }
        dseg.release();
    }
};

struct ppg_pairs {
    int device = -1;
    int32_t rank = 0, nranks = 1;
    int64_t local[2] = {0, 0}, start[2] = {0, 0};   // deduplicated records of this rank / before it
    std::vector<int64_t> dp[2];                     // D[t] - t of the sorted duplicate positions
    std::vector<int64_t> st[2];                     // N ranks: deduplicated records before rank r (r = 0..R)
    PairEmit em;
    ppg_pair_result res{};
    bool checked = false;
    // device scratch, kept across checks (grow only)
    DevBuf<int64_t> keys[2];                        // extracted keys (one-batch shards without set_keys)
    DevBuf<int64_t> dkeys[2];                       // deduplicated keys this rank sends
    DevBuf<int64_t> own[2];                         // keys of the pairs this rank owns
    DevBuf<uint64_t> dpos;
    DevBuf<int64_t> ddp;
    DevBuf<uint32_t> dcount;
    DevBuf<unsigned long long> dres;
    void release() {
        for (int f = 0; f < 2; f++) { keys[f].release(); dkeys[f].release(); own[f].release(); }
        em.release();
        dpos.release();
        ddp.release();
        dcount.release();
        dres.release();
    }
};

namespace {

template <class B>
hipError_t grow(B &b, size_t need) {
    if (b.p && b.n >= need) return hipSuccess;
    return b.alloc(std::max(need, b.n + b.n / 2));
}

unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(8192, (n + 255) / 256)); }

// The shard's spot keys on the device: the set_keys buffer its last run filled, or extracted now
// (one-batch shards); the duplicates' map into p->dp[f]
int local_keys(ppg_pairs *p, int f, ppg_shard *sh, hipStream_t s, const int64_t *&keys, int64_t &n) {
    if (!sh || !sh->ran || sh->last_rc != PPG_OK) return PPG_ARG_ERROR;
    n = sh->total_records;
    if (sh->keys_dev && sh->keys_written) {
        keys = sh->keys_dev;
    } else if (sh->batches.size() == 1) {
        HIPCHK(grow(p->keys[f], (size_t)std::max<int64_t>(n, 1)));
        HIPCHK(ppg_launch_record_keys(s, sh->out.p, sh->jobs.p, sh->res.p, sh->offs.p, sh->oref.p, sh->info.p,
                                      sh->base.p, sh->recs.p, p->keys[f].p, sh->n));
        keys = p->keys[f].p;
    } else {
        return PPG_ARG_ERROR;   // a multi-batch shard's output is gone: its keys needed ppg_shard_set_keys
    }
    // Q1 duplicates: at most one per chunk (a chunk's first record when it lies inside the offset)
    const uint32_t cap = (uint32_t)sh->n + 16;
    HIPCHK(grow(p->dpos, cap));
    HIPCHK(grow(p->dcount, 1));
    HIPCHK(hipMemsetAsync(p->dcount.p, 0, 4, s));
    if (n) hipLaunchKernelGGL(ppg_key_dups, dim3(grid_for((uint64_t)n)), dim3(256), 0, s, keys, (uint64_t)n, p->dpos.p,
                              cap, p->dcount.p);
    HIPCHK(hipGetLastError());
    uint32_t nd = 0;
    HIPCHK(hipMemcpyAsync(&nd, p->dcount.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nd > cap) return PPG_DATA_ERROR;
    std::vector<uint64_t> pos(nd);
    if (nd) HIPCHK(hipMemcpy(pos.data(), p->dpos.p, 8 * (size_t)nd, hipMemcpyDeviceToHost));
    std::sort(pos.begin(), pos.end());
    p->dp[f].resize(nd);
    for (uint32_t t = 0; t < nd; t++) p->dp[f][t] = (int64_t)pos[t] - (int64_t)t;
    p->res.duplicates[f] = nd;
    p->local[f] = n - nd;
    return PPG_OK;
}

// deduplicated numbers [lo, lo + m) of file f's local keys into dst
int compact(ppg_pairs *p, int f, const int64_t *keys, int64_t lo, int64_t m, int64_t *dst, hipStream_t s) {
    if (m <= 0) return PPG_OK;
    const uint32_t nd = (uint32_t)p->dp[f].size();
    HIPCHK(grow(p->ddp, std::max<size_t>(nd, 1)));
    if (nd) HIPCHK(hipMemcpyAsync(p->ddp.p, p->dp[f].data(), 8 * (size_t)nd, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(ppg_key_compact, dim3((unsigned)((m + kCompactSpan - 1) / kCompactSpan)), dim3(256), 0, s, keys,
                       p->ddp.p, nd, (uint64_t)lo, (uint64_t)m, dst);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // ddp is reused by the next call
    return PPG_OK;
}

// mismatches of a vs b over [0, n); first mismatch index and its keys
int compare(ppg_pairs *p, const int64_t *a, const int64_t *b, int64_t n, hipStream_t s, int64_t &mism, int64_t &first,
            int64_t &ka, int64_t &kb) {
    mism = 0;
    first = -1;
    ka = kb = -1;
    if (n <= 0) return PPG_OK;
    HIPCHK(grow(p->dres, 2));
    const unsigned long long init[2] = {0ull, ~0ull};
    HIPCHK(hipMemcpyAsync(p->dres.p, init, sizeof init, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(ppg_pair_compare, dim3(grid_for((uint64_t)n)), dim3(256), 0, s, a, b, (uint64_t)n, p->dres.p);
    HIPCHK(hipGetLastError());
    unsigned long long r[2];
    HIPCHK(hipMemcpyAsync(r, p->dres.p, sizeof r, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    mism = (int64_t)r[0];
    if (mism) {
        first = (int64_t)r[1];
        HIPCHK(hipMemcpy(&ka, a + first, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&kb, b + first, 8, hipMemcpyDeviceToHost));
    }
    return PPG_OK;
}

// the check on one rank (no comm): both files' deduplicated keys compared where they are
int check_local(ppg_pairs *p, const int64_t *k[2], hipStream_t s) {
    ppg_pair_result &R = p->res;
    const int64_t pairs = std::min(p->local[0], p->local[1]);
    const int64_t *cmp[2];
    for (int f = 0; f < 2; f++) {
        if (p->dp[f].empty()) {
            cmp[f] = k[f];
        } else {
            HIPCHK(grow(p->dkeys[f], (size_t)std::max<int64_t>(pairs, 1)));
            if (int rc = compact(p, f, k[f], 0, pairs, p->dkeys[f].p, s)) return rc;
            cmp[f] = p->dkeys[f].p;
        }
    }
    int64_t mism, first, ka, kb;
    if (int rc = compare(p, cmp[0], cmp[1], pairs, s, mism, first, ka, kb)) return rc;
    R.pairs = pairs;
    R.records[0] = p->local[0];
    R.records[1] = p->local[1];
    R.mismatches = mism + std::abs(p->local[0] - p->local[1]);
    R.first_bad = mism ? first : (R.mismatches ? pairs : -1);
    R.first_keys[0] = mism ? ka : -1;
    R.first_keys[1] = mism ? kb : -1;
    return PPG_OK;
}

}  // namespace

// the multi-rank check (every rank calls it; every rank always joins both gathers and the exchange)
static int check_dist(ppg_pairs *p, ppg_comm *comm, const int64_t *k[2], int status, hipStream_t s) {
    const int32_t R = p->nranks, me = p->rank;
    // phase 1: every rank's status and deduplicated counts
    int64_t mine[3] = {status, p->local[0], p->local[1]};
    std::vector<int64_t> all(3 * (size_t)R, 0);
    bool sent_ok = true;
    if (int rc = comm_all_gather_i64(comm, mine, all.data(), 3, sent_ok)) return rc;
    for (int32_t r = 0; r < R; r++)
        if (all[3 * (size_t)r] != PPG_OK) return (int)all[3 * (size_t)r];
    if (!sent_ok) return PPG_DEVICE_ERROR;
    int64_t tot[2] = {0, 0};
    std::vector<int64_t> st[2] = {std::vector<int64_t>((size_t)R + 1, 0), std::vector<int64_t>((size_t)R + 1, 0)};
    for (int f = 0; f < 2; f++)
        for (int32_t r = 0; r < R; r++) st[f][(size_t)r + 1] = st[f][(size_t)r] + all[3 * (size_t)r + 1 + f];
    tot[0] = st[0][(size_t)R];
    tot[1] = st[1][(size_t)R];
    const int64_t pairs = std::min(tot[0], tot[1]);
    std::vector<int64_t> own((size_t)R + 1);
    for (int32_t r = 0; r <= R; r++) own[(size_t)r] = (int64_t)((__int128)pairs * r / R);
    p->start[0] = st[0][(size_t)me];
    p->start[1] = st[1][(size_t)me];
    p->st[0] = st[0];
    p->st[1] = st[1];
    const int64_t mine_pairs = own[(size_t)me + 1] - own[(size_t)me];
    // phase 2: every key to the rank that owns its pair number, one all-to-all-v per file (the keys
    // a rank sends are its deduplicated ones below `pairs`, compacted first; every rank agrees that
    // every rank is ready before any exchange starts)
    std::vector<int64_t> m[2];
    int rc = PPG_OK;
    for (int f = 0; f < 2; f++) {
        m[f].assign((size_t)R * R, 0);
        for (int32_t a = 0; a < R; a++)
            for (int32_t b = 0; b < R; b++)
                m[f][(size_t)a * R + b] = std::max<int64_t>(0, std::min(st[f][(size_t)a + 1], own[(size_t)b + 1]) -
                                                                   std::max(st[f][(size_t)a], own[(size_t)b]));
        const int64_t send = std::max<int64_t>(0, std::min(p->local[f], pairs - p->start[f]));
        if (rc == PPG_OK && (grow(p->dkeys[f], (size_t)std::max<int64_t>(send, 1)) != hipSuccess ||
                             grow(p->own[f], (size_t)std::max<int64_t>(mine_pairs, 1)) != hipSuccess))
            rc = PPG_MEM_ERROR;
        if (rc == PPG_OK) rc = compact(p, f, k[f], 0, send, p->dkeys[f].p, s);
    }
    {
        int64_t st1 = rc;
        std::vector<int64_t> v((size_t)R, 0);
        if (int g = comm_all_gather_i64(comm, &st1, v.data(), 1, sent_ok)) return g;
        for (int32_t r = 0; r < R; r++)
            if (v[(size_t)r] != PPG_OK) return (int)v[(size_t)r];
        if (!sent_ok) return PPG_DEVICE_ERROR;
    }
    for (int f = 0; f < 2; f++) {
        const int x = comm_alltoallv_i64(comm, s, p->dkeys[f].p, p->own[f].p, m[f].data(), true);
        if (rc == PPG_OK) rc = x;
    }
    // phase 3: the owned pairs compared, results gathered
    int64_t mism = 0, first = -1, ka = -1, kb = -1;
    if (rc == PPG_OK) rc = compare(p, p->own[0].p, p->own[1].p, mine_pairs, s, mism, first, ka, kb);
    int64_t res[5] = {rc, mism, first >= 0 ? own[(size_t)me] + first : -1, ka, kb};
    std::vector<int64_t> rall(5 * (size_t)R, 0);
    if (int g = comm_all_gather_i64(comm, res, rall.data(), 5, sent_ok)) return g;
    for (int32_t r = 0; r < R; r++)
        if (rall[5 * (size_t)r] != PPG_OK) return (int)rall[5 * (size_t)r];
    ppg_pair_result &Rz = p->res;
    Rz.pairs = pairs;
    Rz.records[0] = tot[0];
    Rz.records[1] = tot[1];
    Rz.mismatches = std::abs(tot[0] - tot[1]);
    Rz.first_bad = -1;
    Rz.first_keys[0] = Rz.first_keys[1] = -1;
    for (int32_t r = 0; r < R; r++) {   // ranks own increasing pair numbers: the first one with a mismatch
        Rz.mismatches += rall[5 * (size_t)r + 1];
        if (Rz.first_bad < 0 && rall[5 * (size_t)r + 1]) {
            Rz.first_bad = rall[5 * (size_t)r + 2];
            Rz.first_keys[0] = rall[5 * (size_t)r + 3];
            Rz.first_keys[1] = rall[5 * (size_t)r + 4];
        }
    }
    if (Rz.first_bad < 0 && Rz.mismatches) Rz.first_bad = pairs;
    return PPG_OK;
}

// ================= record-aligned pair chunks (ppg_pairs_emit_*, include/ppgpu.h) =================
namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// Test hook (tests only), in the style of PPG_IX_PERTURB: PPG_PAIRS_PERTURB=short
// takes one pair chunk off the last output batch's deduplicated record range (so no batch can ever
// complete the last pair chunks: the no-progress guards of emit_next_local / emit_next_fused must
// end the emission), =bases leaves make_segs without record bases (every segment search fails).
// A guard that fires under the hook says so on stderr, so a test can tell which one ended it.
int pairs_perturb() {
    const char *e = getenv("PPG_PAIRS_PERTURB");
    if (!e) return 0;
    return !strcmp(e, "short") ? 1 : !strcmp(e, "bases") ? 2 : 0;
}
void guard_note(const char *where) {
    if (pairs_perturb()) fprintf(stderr, "[ppg_pairs] PPG_DATA_ERROR at %s\n", where);
}

// A pair chunk half's descriptors are u32 positions relative to the half (ppg_pack_segs), so a half
// must stay below 4 GiB: longer halves are refused with PPG_UNSUPPORTED before packing.
// PPG_PAIR_HALF_MAX (tests only) lowers the limit so small inputs reach the refusal.
int64_t half_max() {
    const char *e = getenv("PPG_PAIR_HALF_MAX");
    const int64_t v = e ? strtoll(e, nullptr, 10) : 0;
    return v > 0 && v < (int64_t)UINT32_MAX ? v : (int64_t)UINT32_MAX;
}

// shard record number of this rank's deduplicated record d (skip the duplicates at or before it)
int64_t shard_rec(const std::vector<int64_t> &dp, int64_t d) {
    return d + (int64_t)(std::upper_bound(dp.begin(), dp.end(), d) - dp.begin());
}
// deduplicated number of the first record at or after shard record r
int64_t dedup_of(const std::vector<int64_t> &pos, int64_t r) {
    return r - (int64_t)(std::lower_bound(pos.begin(), pos.end(), r) - pos.begin());
}

// where a segment of records lands: the segment list is built first, placed once their byte spans are known
struct SegPlace {
    int32_t grp;        // destination group (a pair chunk half, or an exchange piece)
};

// The runs of consecutive records of this rank's deduplicated records [d0, d1) of file f, split at
// chunk boundaries and at the duplicates, from the shard's resident output batch
// (false: the records are not where the shard's run put them -- never expected; the caller fails
// with PPG_DATA_ERROR instead of looping)
bool make_segs(const ppg_pairs *p, int f, int64_t d0, int64_t d1, int32_t grp, std::vector<PpgPackSeg> &seg,
               std::vector<SegPlace> &pl) {
    const PairEmit &E = p->em;
    const ppg_shard *sh = E.sh[f];
    const auto &B = sh->h_base;
    // chunks whose record bases are set (emit_run: the batches run so far; the rest are still 0)
    const auto Bend = B.begin() + std::min<std::ptrdiff_t>((std::ptrdiff_t)B.size(), pairs_perturb() == 2 ? 0 : E.kvalid[f]);
    const auto &pos = E.pos[f];
    int64_t d = d0;
    while (d < d1) {
        const int64_t r = shard_rec(p->dp[f], d);
        const int32_t k = (int32_t)(std::upper_bound(B.begin(), Bend, r) - B.begin()) - 1;
        if (k < 0) { guard_note("make_segs (no chunk with a record base holds the record)"); return false; }
        const int64_t cend = B[(size_t)k] + (int64_t)sh->h_info[(size_t)k].records;
        const auto nd = std::upper_bound(pos.begin(), pos.end(), r);
        const int64_t stop = std::min<int64_t>(cend, nd == pos.end() ? INT64_MAX : *nd);
        const int64_t run = std::min(stop - r, d1 - d);
        if (run <= 0) { guard_note("make_segs (no progress)"); return false; }
        const PpgInflateJob &J = sh->h_jobs[(size_t)k];
        PpgPackSeg g{};
        g.off = sh->offs.p + E.offst[f][(size_t)k];
        g.olen = J.raw_shift;
        g.body = sh->out.p + J.out_off;
        g.desc = sh->recs.p + 4 * r;
        g.nrec = (uint32_t)run;
        g.first = r == B[(size_t)k] ? 1u : 0u;
        seg.push_back(g);
        pl.push_back(SegPlace{grp});
        d += run;
    }
    return true;
}

template <class B>
int grow_keep(B &b, size_t need, hipStream_t s, size_t keep) {   // grow, keeping the first `keep` elements
    if (b.p && b.n >= need) return PPG_OK;
    B g;
    HIPCHK(g.alloc(std::max(need, b.n + b.n / 2)));
    if (keep) HIPCHK(hipMemcpyAsync(g.p, b.p, keep * sizeof(*b.p), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    std::swap(g.p, b.p);
    std::swap(g.n, b.n);
    return PPG_OK;
}

// fill a, b of every segment (their first and last records' descriptors), on the device
int seg_bounds(PairEmit &E, std::vector<PpgPackSeg> &seg, hipStream_t s) {
    if (seg.empty()) return PPG_OK;
    HIPCHK(grow(E.dseg, seg.size()));
    HIPCHK(hipMemcpyAsync(E.dseg.p, seg.data(), sizeof(PpgPackSeg) * seg.size(), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(ppg_seg_bounds, dim3((unsigned)((seg.size() + 255) / 256)), dim3(256), 0, s, E.dseg.p, (int)seg.size());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(seg.data(), E.dseg.p, sizeof(PpgPackSeg) * seg.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return PPG_OK;
}

// copy the placed segments (dst, ddst, delta set) into dst / ddesc
int seg_pack(PairEmit &E, const std::vector<PpgPackSeg> &seg, uint8_t *dst, uint32_t *ddesc, hipStream_t s) {
    if (seg.empty()) return PPG_OK;
    HIPCHK(grow(E.dseg, seg.size()));
    HIPCHK(hipMemcpyAsync(E.dseg.p, seg.data(), sizeof(PpgPackSeg) * seg.size(), hipMemcpyHostToDevice, s));
    uint64_t mx = 0;
    for (const auto &g : seg) mx = std::max<uint64_t>(mx, g.b - g.a);
    const unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, mx / 65536 + 1));
    const unsigned gy = (unsigned)std::min<size_t>(seg.size(), 65535);
    hipLaunchKernelGGL(ppg_pack_segs, dim3(gx, gy), dim3(256), 0, s, E.dseg.p, (int)seg.size(), dst, ddesc);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // the host segment list and dseg are reused
    return PPG_OK;
}

// batch b of a shard's batches run again, its output resident (one rank: the windows advance over
// the batches): launch, then collect (two shards' batches are in flight together); the shard's
// record totals, bases, keys and timing are left as its run left them
int rerun_launch(ppg_shard *sh, int32_t b, RerunSave &sv) {
    const auto [b0, b1] = sh->batches[(size_t)b];
    sv = RerunSave{sh->total_records, sh->t_inflate, sh->t_parse, sh->t_total, sh->keys_dev};
    sh->total_records = sh->h_base[(size_t)b0];   // descriptors rewritten where the run wrote them
    sh->keys_dev = nullptr;
    const int rc = batch_launch(sh, b0, b1);
    if (rc != PPG_OK) {
        sh->total_records = sv.tot;
        sh->keys_dev = sv.keys;
    }
    return rc;
}

int rerun_collect(ppg_shard *sh, int32_t b, const RerunSave &sv) {
    const auto [b0, b1] = sh->batches[(size_t)b];
    float ms = 0;
    const int rc = batch_collect(sh, b0, b1, ms);
    sh->total_records = sv.tot;
    sh->t_inflate = sv.ti;
    sh->t_parse = sv.tp;
    sh->t_total = sv.tt;
    sh->keys_dev = sv.keys;
    return rc;
}

// Steps 2-3 of a one-rank window: pair chunks [e, J) are complete in both files' resident batches
// (pairs: the pair count, or a bound below which every pair chunk < J is final); the window is cut
// at the byte budget, then both files' halves are placed and packed
int pack_window(ppg_pairs *p, int64_t e, int64_t J, int64_t pairs, Clock::time_point t0, int64_t *j0, int64_t *j1) {
    PairEmit &E = p->em;
    const int64_t K = E.K;
    if (J <= e) return PPG_DATA_ERROR;
    const auto tp = Clock::now();
    std::vector<PpgPackSeg> seg[2];
    std::vector<SegPlace> pl[2];
    for (int f = 0; f < 2; f++) {
        for (int64_t j = e; j < J; j++) {
            const int64_t a = j == e ? e * K + E.cnrec[f] : j * K, z = std::min((j + 1) * K, pairs);
            if (!make_segs(p, f, a, z, (int32_t)(j - e), seg[f], pl[f])) return PPG_DATA_ERROR;
        }
        if (int rc = seg_bounds(E, seg[f], shard_stream(E.sh[f]))) return rc;
    }
    // cut the window where either file's halves pass the byte budget (one pair chunk at least)
    std::vector<int64_t> hb[2];
    for (int f = 0; f < 2; f++) {
        hb[f].assign((size_t)(J - e), 0);
        hb[f][0] = E.clen[f];
        for (size_t i = 0; i < seg[f].size(); i++) hb[f][(size_t)pl[f][i].grp] += (int64_t)(seg[f][i].b - seg[f][i].a);
    }
    int64_t J2 = e + 1;
    {
        int64_t acc[2] = {(hb[0][0] + 15) / 16 * 16, (hb[1][0] + 15) / 16 * 16};
        while (J2 < J) {
            const size_t i = (size_t)(J2 - e);
            if (acc[0] + hb[0][i] > E.window_bytes || acc[1] + hb[1][i] > E.window_bytes) break;
            acc[0] += (hb[0][i] + 15) / 16 * 16;
            acc[1] += (hb[1][i] + 15) / 16 * 16;
            J2++;
        }
    }
    // a half's descriptors are u32 positions relative to it (ppg_pack_segs)
    for (int f = 0; f < 2; f++)
        for (int64_t i = 0; i < J2 - e; i++)
            if (hb[f][(size_t)i] > half_max()) return PPG_UNSUPPORTED;
    // 3. place and pack both files' halves of pair chunks [e, J2)
    for (int f = 0; f < 2; f++) {
        hipStream_t s = shard_stream(E.sh[f]);
        const size_t nj = (size_t)(J2 - e);
        E.boff[f].assign(nj, 0);
        E.blen[f].assign(nj, 0);
        E.roff[f].assign(nj, 0);
        E.rcnt[f].assign(nj, 0);
        int64_t bo = 0, ro = 0;
        for (size_t i = 0; i < nj; i++) {
            E.boff[f][i] = bo;
            E.roff[f][i] = ro;
            E.blen[f][i] = hb[f][i];
            const int64_t lo = i == 0 ? e * K : (e + (int64_t)i) * K, z = std::min((e + (int64_t)i + 1) * K, pairs);
            E.rcnt[f][i] = z - lo;
            bo += (hb[f][i] + 15) / 16 * 16;
            ro += E.rcnt[f][i];
        }
        if (int rc = grow_keep(E.bytes[f], (size_t)bo + 64, s, 0)) return rc;
        if (int rc = grow_keep(E.desc[f], 4 * (size_t)ro + 4, s, 0)) return rc;
        // the carried first part of pair chunk e (its descriptors are relative to the half already)
        if (E.cnrec[f]) {
            HIPCHK(hipMemcpyAsync(E.bytes[f].p, E.cbytes[f].p, (size_t)E.clen[f], hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(E.desc[f].p, E.cdesc[f].p, 16 * (size_t)E.cnrec[f], hipMemcpyDeviceToDevice, s));
        }
        std::vector<int64_t> at(nj, 0), rat(nj, 0);
        at[0] = E.clen[f];
        rat[0] = E.cnrec[f];
        std::vector<PpgPackSeg> go;
        for (size_t i = 0; i < seg[f].size(); i++) {
            const size_t g = (size_t)pl[f][i].grp;
            if (g >= nj) break;
            PpgPackSeg x = seg[f][i];
            x.dst = (uint64_t)(E.boff[f][g] + at[g]);
            x.ddst = (uint64_t)(E.roff[f][g] + rat[g]);
            x.delta = at[g] - (int64_t)x.a;
            at[g] += (int64_t)(x.b - x.a);
            rat[g] += x.nrec;
            go.push_back(x);
        }
        if (int rc = seg_pack(E, go, E.bytes[f].p, E.desc[f].p, s)) return rc;
        E.clen[f] = E.cnrec[f] = 0;
    }
    E.t_ms[1] += ms_since(tp);
    E.w0 = e;
    E.w1 = J2;
    E.next = J2;
    E.t_ms[3] += ms_since(t0);
    if (j0) *j0 = e;
    if (j1) *j1 = J2;
    return PPG_OK;
}

// A resident batch b holding only the first part of the current pair chunk's half (records from
// cend on): that part goes to the carry before the next batch's run overwrites the output
int carry_rest(ppg_pairs *p, int f, int64_t cend, int32_t b) {
    PairEmit &E = p->em;
    if (b < 0 || !(E.blo[f][(size_t)b] <= cend && cend < E.bhi[f][(size_t)b])) return PPG_OK;
    hipStream_t s = shard_stream(E.sh[f]);
    std::vector<PpgPackSeg> seg;
    std::vector<SegPlace> pl;
    if (!make_segs(p, f, cend, E.bhi[f][(size_t)b], 0, seg, pl)) return PPG_DATA_ERROR;
    if (int rc = seg_bounds(E, seg, s)) return rc;
    int64_t add = 0, nadd = 0;
    for (auto &g : seg) {
        g.dst = (uint64_t)(E.clen[f] + add);
        g.ddst = (uint64_t)(E.cnrec[f] + nadd);
        g.delta = (int64_t)g.dst - (int64_t)g.a;   // the carry starts its half
        add += (int64_t)(g.b - g.a);
        nadd += g.nrec;
    }
    if (E.clen[f] + add > half_max()) return PPG_UNSUPPORTED;   // the carry starts a half (u32 descriptors)
    if (int rc = grow_keep(E.cbytes[f], (size_t)(E.clen[f] + add) + 64, s, (size_t)E.clen[f])) return rc;
    if (int rc = grow_keep(E.cdesc[f], 4 * (size_t)(E.cnrec[f] + nadd) + 4, s, 4 * (size_t)E.cnrec[f])) return rc;
    if (int rc = seg_pack(E, seg, E.cbytes[f].p, E.cdesc[f].p, s)) return rc;
    E.clen[f] += add;
    E.cnrec[f] += nadd;
    return PPG_OK;
}

// ---- one rank: windows over the shards' batches ----
int emit_next_local(ppg_pairs *p, int64_t *j0, int64_t *j1) {
    PairEmit &E = p->em;
    const int64_t K = E.K, pairs = p->res.pairs, e = E.next;
    if (e >= E.j_hi) return PPG_STREAM_END;
    const auto t0 = Clock::now();
    // 1. each file's resident batch must complete pair chunk e; a batch holding only its first part
    //    hands that part to the carry first (the next batch's run overwrites the output).  Both
    //    files' batches run together, each on its shard's own stream.
    const int64_t need = std::min((e + 1) * K, pairs);
    for (;;) {
        bool run[2] = {false, false};
        for (int f = 0; f < 2; f++) {
            ppg_shard *sh = E.sh[f];
            const int64_t cend = e * K + E.cnrec[f];
            const int32_t b = E.batch[f];
            if (E.blo[f][(size_t)b] <= cend && E.bhi[f][(size_t)b] >= need) continue;
            if (int rc = carry_rest(p, f, cend, b)) return rc;
            (void)sh;
            // the batch holding the carry's end
            const int64_t c2 = e * K + E.cnrec[f];
            int32_t nb = 0;
            while ((size_t)nb + 1 < E.bhi[f].size() && E.bhi[f][(size_t)nb] <= c2) nb++;
            if (nb == b) {   // no progress: the batches cannot complete the pair chunk
                guard_note("emit_next_local (no batch completes the pair chunk)");
                return PPG_DATA_ERROR;
            }
            E.batch[f] = nb;
            run[f] = true;
        }
        if (!run[0] && !run[1]) break;
        const auto tr = Clock::now();
        int rc = PPG_OK;
        bool launched[2] = {false, false};
        for (int f = 0; f < 2 && rc == PPG_OK; f++)
            if (run[f]) {
                rc = rerun_launch(E.sh[f], E.batch[f], E.save[f]);
                launched[f] = rc == PPG_OK;
            }
        for (int f = 0; f < 2; f++)
            if (launched[f]) {
                const int x = rerun_collect(E.sh[f], E.batch[f], E.save[f]);
                if (rc == PPG_OK) rc = x;
            }
        if (rc != PPG_OK) return rc;
        E.reruns += run[0] + run[1];
        E.t_ms[0] += ms_since(tr);
    }
    // 2. the window: the pair chunks both resident batches complete, within the byte budget
    int64_t J = E.j_hi;
    for (int f = 0; f < 2; f++) {
        const int64_t hi = E.bhi[f][(size_t)E.batch[f]];
        if (hi < pairs) J = std::min(J, hi / K);
    }
    return pack_window(p, e, J, pairs, t0, j0, j1);
}

// ---- one rank, fused (ppg_pairs_emit_run): the shards' first run, driven by the windows ----
// Batch b of file f has just run for the first time: its chunks' parse info, the duplicates among
// its records (ppg_key_dups over its keys; SURVEY Q1: at most one per chunk, so the numbering map
// grows batch by batch), its deduplicated record range; after the file's last batch the shard is
// finished exactly as ppg_shard_run leaves it (results, status, keys marked written).
int fused_collected(ppg_pairs *p, int f, int32_t b) {
    PairEmit &E = p->em;
    ppg_shard *sh = E.sh[f];
    hipStream_t s = shard_stream(sh);
    const auto [b0, b1] = sh->batches[(size_t)b];
    const int64_t r0 = sh->h_base[(size_t)b0], r1 = sh->total_records;
    sh->h_info.resize((size_t)sh->n);
    if (b1 > b0)
        HIPCHK(hipMemcpyAsync(sh->h_info.data() + b0, sh->info.p + b0, sizeof(PpgParseInfo) * (size_t)(b1 - b0),
                              hipMemcpyDeviceToHost, s));
    const uint32_t cap = (uint32_t)(b1 - b0) + 16;
    HIPCHK(grow(p->dpos, cap));
    HIPCHK(grow(p->dcount, 1));
    HIPCHK(hipMemsetAsync(p->dcount.p, 0, 4, s));
    if (r1 > r0)
        hipLaunchKernelGGL(ppg_key_dups, dim3(grid_for((uint64_t)(r1 - r0))), dim3(256), 0, s, sh->keys_dev + r0,
                           (uint64_t)(r1 - r0), p->dpos.p, cap, p->dcount.p);
    HIPCHK(hipGetLastError());
    uint32_t nd = 0;
    HIPCHK(hipMemcpyAsync(&nd, p->dcount.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nd > cap) return PPG_DATA_ERROR;
    std::vector<uint64_t> pos(nd);
    if (nd) HIPCHK(hipMemcpy(pos.data(), p->dpos.p, 8 * (size_t)nd, hipMemcpyDeviceToHost));
    std::sort(pos.begin(), pos.end());
    for (uint64_t x : pos) {
        const int64_t r = r0 + (int64_t)x;
        p->dp[f].push_back(r - (int64_t)E.pos[f].size());
        E.pos[f].push_back(r);
    }
    E.blo[f].push_back(dedup_of(E.pos[f], r0));
    E.bhi[f].push_back(dedup_of(E.pos[f], r1));
    if (pairs_perturb() == 1 && (size_t)b + 1 == sh->batches.size())
        E.bhi[f].back() = std::max(E.blo[f].back(), E.bhi[f].back() - E.K);
    E.kvalid[f] = b1;
    if ((size_t)b + 1 == sh->batches.size()) {
        const int rc = shard_finish(sh, E.run_ms[f]);
        sh->last_rc = rc;
        sh->keys_written = rc == PPG_OK && sh->keys_dev != nullptr;
        if (rc != PPG_OK) return rc;
        E.done[f] = true;
        p->local[f] = sh->total_records - (int64_t)E.pos[f].size();
    }
    return PPG_OK;
}

// the next batch of the files in run[] (first runs, both in flight together)
int fused_run(ppg_pairs *p, const bool run[2]) {
    PairEmit &E = p->em;
    const auto tr = Clock::now();
    int rc = PPG_OK;
    bool launched[2] = {false, false};
    for (int f = 0; f < 2 && rc == PPG_OK; f++)
        if (run[f]) {
            ppg_shard *sh = E.sh[f];
            const int32_t b = ++E.batch[f];
            rc = batch_launch(sh, sh->batches[(size_t)b].first, sh->batches[(size_t)b].second);
            launched[f] = rc == PPG_OK;
        }
    for (int f = 0; f < 2; f++)
        if (launched[f]) {
            ppg_shard *sh = E.sh[f];
            const int32_t b = E.batch[f];
            int x = batch_collect(sh, sh->batches[(size_t)b].first, sh->batches[(size_t)b].second, E.run_ms[f]);
            if (x == PPG_OK) x = fused_collected(p, f, b);
            if (x != PPG_OK) sh->last_rc = x;
            if (rc == PPG_OK) rc = x;
        }
    E.t_ms[0] += ms_since(tr);
    return rc;
}

// pairs known so far: the smaller finished file's deduplicated count bounds them (INT64_MAX: neither)
int64_t fused_bound(const ppg_pairs *p) {
    int64_t b = INT64_MAX;
    for (int f = 0; f < 2; f++)
        if (p->em.done[f]) b = std::min(b, p->local[f]);
    return b;
}

int emit_next_fused(ppg_pairs *p, int64_t *j0, int64_t *j1) {
    PairEmit &E = p->em;
    const int64_t K = E.K, e = E.next;
    const auto t0 = Clock::now();
    for (;;) {
        const int64_t bound = fused_bound(p);
        if (bound != INT64_MAX && e * K >= bound) {
            // no pair chunk left: the unfinished file's remaining batches still run (the shards end
            // as ppg_shard_run leaves them, for ppg_pairs_check and the shards' own results)
            for (int f = 0; f < 2; f++)
                while (!E.done[f]) {
                    const bool run[2] = {f == 0, f == 1};
                    if (int rc = fused_run(p, run)) return rc;
                }
            E.npc = (std::min(p->local[0], p->local[1]) + K - 1) / K;
            E.j_hi = E.npc;
            return PPG_STREAM_END;
        }
        // 1. each file's resident batch must complete pair chunk e (the first part carried over when
        //    the batch holds only that); else its next batch runs
        const int64_t need = std::min((e + 1) * K, bound);
        bool run[2] = {false, false};
        for (int f = 0; f < 2; f++) {
            const int64_t cend = e * K + E.cnrec[f];
            const int32_t b = E.batch[f];
            if (b >= 0 && E.blo[f][(size_t)b] <= cend && E.bhi[f][(size_t)b] >= need) continue;
            if (E.done[f]) {   // every batch has run and the pair chunk is not complete
                guard_note("emit_next_fused (every batch has run, the pair chunk is incomplete)");
                return PPG_DATA_ERROR;
            }
            if (int rc = carry_rest(p, f, cend, b)) return rc;
            run[f] = true;
        }
        if (!run[0] && !run[1]) break;
        if (int rc = fused_run(p, run)) return rc;
    }
    // 2. the window: what both resident batches complete (a finished file's last batch reaches its
    //    end; the pair count is final once both have finished, bounded by a finished file's before)
    const int64_t bound = fused_bound(p);
    int64_t J = bound == INT64_MAX ? INT64_MAX : (bound + K - 1) / K;
    for (int f = 0; f < 2; f++)
        if (!(E.done[f] && (size_t)E.batch[f] + 1 == E.sh[f]->batches.size()))
            J = std::min(J, E.bhi[f][(size_t)E.batch[f]] / K);
    return pack_window(p, e, J, bound, t0, j0, j1);
}

// ---- N ranks: one window, the records this rank does not hold moved over the comm ----
int emit_exchange(ppg_pairs *p, int64_t *j0, int64_t *j1) {
    PairEmit &E = p->em;
    const int32_t R = p->nranks, me = p->rank;
    const int64_t K = E.K, pairs = p->res.pairs;
    const auto t0 = Clock::now();
    // ownership: rank r owns the pair chunks that start in its R1 range
    std::vector<int64_t> jr((size_t)R + 1);
    for (int32_t r = 0; r < R; r++) jr[(size_t)r] = std::min(E.npc, (p->st[0][(size_t)r] + K - 1) / K);
    jr[(size_t)R] = E.npc;
    for (int32_t r = 1; r <= R; r++) jr[(size_t)r] = std::max(jr[(size_t)r], jr[(size_t)r - 1]);
    auto own_lo = [&](int32_t r) { return std::min(jr[(size_t)r] * K, pairs); };
    auto own_hi = [&](int32_t r) { return std::min(jr[(size_t)r + 1] * K, pairs); };
    E.j_lo = jr[(size_t)me];
    E.j_hi = jr[(size_t)me + 1];
    int status = PPG_OK;
    hipStream_t s = shard_stream(E.sh[0]);
    // 1. this rank's records to each owner: one piece per (owner, pair chunk), packed by owner
    std::vector<int64_t> sendw[2];   // per owner: int64 words of bytes
    std::vector<int64_t> piece_len[2];
    for (int f = 0; f < 2 && status == PPG_OK; f++) {
        sendw[f].assign((size_t)R, 0);
        const int64_t h0 = p->st[f][(size_t)me], h1 = p->st[f][(size_t)me + 1];
        std::vector<PpgPackSeg> seg;
        std::vector<SegPlace> pl;
        std::vector<int32_t> pdst;   // owner of each piece
        int32_t np = 0;
        for (int32_t r = 0; r < R && status == PPG_OK; r++) {
            const int64_t a = std::max(h0, own_lo(r)), z = std::min(h1, own_hi(r));
            for (int64_t lo = a; lo < z;) {
                const int64_t hi = std::min(z, (lo / K + 1) * K);
                if (!make_segs(p, f, lo - h0, hi - h0, np++, seg, pl)) {
                    status = PPG_DATA_ERROR;
                    break;
                }
                pdst.push_back(r);
                lo = hi;
            }
        }
        if (status != PPG_OK) break;
        status = seg_bounds(E, seg, s);
        if (status != PPG_OK) break;
        piece_len[f].assign((size_t)np, 0);
        std::vector<int64_t> piece_rec((size_t)np, 0);
        for (size_t i = 0; i < seg.size(); i++) {
            piece_len[f][(size_t)pl[i].grp] += (int64_t)(seg[i].b - seg[i].a);
            piece_rec[(size_t)pl[i].grp] += seg[i].nrec;
        }
        for (int64_t L : piece_len[f])   // a piece lies in one half (u32 descriptors): joins the status gather
            if (L > half_max()) status = PPG_UNSUPPORTED;
        if (status != PPG_OK) break;
        // owner groups: pieces back to back, each group padded to 8 bytes (int64 words)
        std::vector<int64_t> poff((size_t)np), proff((size_t)np);
        int64_t gb = 0, gr = 0;
        for (int32_t r = 0, i = 0; r < R; r++) {
            const int64_t start = gb;
            for (; i < np && pdst[(size_t)i] == r; i++) {
                poff[(size_t)i] = gb;
                proff[(size_t)i] = gr;
                gb += piece_len[f][(size_t)i];
                gr += piece_rec[(size_t)i];
            }
            gb = (gb + 7) / 8 * 8;
            sendw[f][(size_t)r] = (gb - start) / 8;
        }
        std::vector<int64_t> at((size_t)np, 0), rat((size_t)np, 0);
        for (size_t i = 0; i < seg.size(); i++) {
            const size_t g = (size_t)pl[i].grp;
            seg[i].dst = (uint64_t)(poff[g] + at[g]);
            seg[i].ddst = (uint64_t)(proff[g] + rat[g]);
            seg[i].delta = at[g] - (int64_t)seg[i].a;   // descriptors relative to their piece
            at[g] += (int64_t)(seg[i].b - seg[i].a);
            rat[g] += seg[i].nrec;
        }
        if (grow(E.sbuf[f], (size_t)gb / 8 + 8) != hipSuccess || grow(E.sdesc[f], 2 * (size_t)gr + 2) != hipSuccess) {
            status = PPG_MEM_ERROR;
            break;
        }
        status = seg_pack(E, seg, (uint8_t *)E.sbuf[f].p, (uint32_t *)E.sdesc[f].p, s);
    }
    // 2. every rank's status and per-owner word counts (both files), then the exchanges
    std::vector<int64_t> mine(1 + 2 * (size_t)R, 0), all((1 + 2 * (size_t)R) * R, 0);
    mine[0] = status;
    for (int f = 0; f < 2; f++)
        for (int32_t r = 0; r < R; r++) mine[1 + (size_t)f * R + r] = sendw[f].empty() ? 0 : sendw[f][(size_t)r];
    bool sent_ok = true;
    const auto tx = Clock::now();
    if (int g = comm_all_gather_i64(E.comm, mine.data(), all.data(), mine.size(), sent_ok)) return g;
    for (int32_t r = 0; r < R; r++)
        if (all[(size_t)r * mine.size()] != PPG_OK) return (int)all[(size_t)r * mine.size()];
    if (!sent_ok) return PPG_DEVICE_ERROR;
    int rc = PPG_OK;
    std::vector<int64_t> mw[2], md[2];
    for (int f = 0; f < 2; f++) {
        mw[f].assign((size_t)R * R, 0);
        md[f].assign((size_t)R * R, 0);
        for (int32_t q = 0; q < R; q++)
            for (int32_t r = 0; r < R; r++) {
                mw[f][(size_t)q * R + r] = all[(size_t)q * mine.size() + 1 + (size_t)f * R + r];
                const int64_t a = std::max(p->st[f][(size_t)q], own_lo(r)), z = std::min(p->st[f][(size_t)q + 1], own_hi(r));
                md[f][(size_t)q * R + r] = 2 * std::max<int64_t>(0, z - a);
            }
        int64_t rw = 0, rdn = 0;
        for (int32_t q = 0; q < R; q++) {
            rw += mw[f][(size_t)q * R + me];
            rdn += md[f][(size_t)q * R + me];
        }
        if (rc == PPG_OK && (grow(E.rbuf[f], (size_t)rw + 8) != hipSuccess || grow(E.rdesc[f], (size_t)rdn + 2) != hipSuccess))
            rc = PPG_MEM_ERROR;
    }
    {   // agree that every rank has its receive buffers before moving anything
        int64_t st1 = rc;
        std::vector<int64_t> v((size_t)R, 0);
        if (int g = comm_all_gather_i64(E.comm, &st1, v.data(), 1, sent_ok)) return g;
        for (int32_t r = 0; r < R; r++)
            if (v[(size_t)r] != PPG_OK) return (int)v[(size_t)r];
        if (!sent_ok) return PPG_DEVICE_ERROR;
    }
    for (int f = 0; f < 2; f++) {
        const int x = comm_alltoallv_i64(E.comm, s, E.sbuf[f].p, E.rbuf[f].p, mw[f].data(), true);
        const int y = comm_alltoallv_i64(E.comm, s, E.sdesc[f].p, E.rdesc[f].p, md[f].data(), true);
        if (rc == PPG_OK) rc = x != PPG_OK ? x : y;
    }
    E.t_ms[2] += ms_since(tx);
    if (rc != PPG_OK) return rc;
    // 3. the received pieces, source by source, into this rank's pair chunk halves
    const int64_t nj = E.j_hi - E.j_lo;
    for (int f = 0; f < 2; f++) {
        std::vector<PpgPackSeg> seg;
        std::vector<int64_t> pj;    // pair chunk (from j_lo) of each piece
        int64_t wq = 0, rq = 0;     // source group starts (words, records)
        for (int32_t q = 0; q < R; q++) {
            const int64_t a = std::max(p->st[f][(size_t)q], own_lo(me)), z = std::min(p->st[f][(size_t)q + 1], own_hi(me));
            int64_t rr = rq;
            for (int64_t lo = a; lo < z;) {
                const int64_t hi = std::min(z, (lo / K + 1) * K);
                PpgPackSeg g{};
                g.desc = (const uint32_t *)E.rdesc[f].p + 4 * rr;
                g.nrec = (uint32_t)(hi - lo);
                g.first = 1;
                g.body = (const uint8_t *)(E.rbuf[f].p + wq);   // + the piece's offset in its group (below)
                seg.push_back(g);
                pj.push_back(lo / K - E.j_lo);
                rr += hi - lo;
                lo = hi;
            }
            wq += mw[f][(size_t)q * R + me];
            rq += md[f][(size_t)q * R + me] / 2;
        }
        if (int x = seg_bounds(E, seg, s)) return x;   // b = the piece's length (a = 0)
        // bodies: pieces of one source group back to back
        {
            const uint8_t *grp = nullptr;
            uint64_t run = 0;
            for (auto &g : seg) {
                if (g.body != grp) { grp = g.body; run = 0; }
                g.body = grp + run;
                run += g.b;
            }
        }
        E.boff[f].assign((size_t)nj, 0);
        E.blen[f].assign((size_t)nj, 0);
        E.roff[f].assign((size_t)nj, 0);
        E.rcnt[f].assign((size_t)nj, 0);
        for (size_t i = 0; i < seg.size(); i++) {
            E.blen[f][(size_t)pj[i]] += (int64_t)seg[i].b;
            E.rcnt[f][(size_t)pj[i]] += seg[i].nrec;
        }
        // (after the exchange, which every rank joined: a refusal here strands no one)
        for (int64_t L : E.blen[f])
            if (L > half_max()) return PPG_UNSUPPORTED;
        int64_t bo = 0, ro = 0;
        for (int64_t j = 0; j < nj; j++) {
            E.boff[f][(size_t)j] = bo;
            E.roff[f][(size_t)j] = ro;
            bo += (E.blen[f][(size_t)j] + 15) / 16 * 16;
            ro += E.rcnt[f][(size_t)j];
        }
        if (grow(E.bytes[f], (size_t)bo + 64) != hipSuccess || grow(E.desc[f], 4 * (size_t)ro + 4) != hipSuccess)
            return PPG_MEM_ERROR;
        std::vector<int64_t> at((size_t)nj, 0), rat((size_t)nj, 0);
        for (size_t i = 0; i < seg.size(); i++) {
            const size_t j = (size_t)pj[i];
            seg[i].dst = (uint64_t)(E.boff[f][j] + at[j]);
            seg[i].ddst = (uint64_t)(E.roff[f][j] + rat[j]);
            seg[i].delta = at[j];
            at[j] += (int64_t)seg[i].b;
            rat[j] += seg[i].nrec;
        }
        if (int x = seg_pack(E, seg, E.bytes[f].p, E.desc[f].p, s)) return x;
    }
    E.w0 = E.j_lo;
    E.w1 = E.j_hi;
    E.next = E.j_hi;
    E.exchanged = true;
    E.t_ms[3] += ms_since(t0);
    if (j0) *j0 = E.w0;
    if (j1) *j1 = E.w1;
    return PPG_OK;
}

}  // namespace

extern "C" {

int ppg_pairs_create(ppg_pairs **out) {
    if (!out) return PPG_ARG_ERROR;
    *out = new ppg_pairs;
    return PPG_OK;
}

void ppg_pairs_free(ppg_pairs *p) {
    if (!p) return;
    if (p->device >= 0) (void)hipSetDevice(p->device);
    p->release();
    delete p;
}

int ppg_pairs_check(ppg_pairs *p, ppg_shard *r1, ppg_shard *r2, ppg_comm *comm, ppg_pair_result *result) {
    if (!p) return PPG_ARG_ERROR;
    p->checked = false;
    p->res = ppg_pair_result{};
    p->start[0] = p->start[1] = 0;
    int32_t rank = 0, nranks = 1;
    if (comm) comm_size(comm, &rank, &nranks);
    p->rank = rank;
    p->nranks = nranks;
    // local keys; a failing rank still joins the collectives (check_dist) with its status
    int status = PPG_OK;
    const int64_t *k[2] = {nullptr, nullptr};
    hipStream_t s = nullptr;
    if (!r1 || !r2 || r1->ctx->device != r2->ctx->device ||
        (comm && comm_device(comm) >= 0 && comm_device(comm) != r1->ctx->device)) {
        status = PPG_ARG_ERROR;
    } else {
        if (p->device != r1->ctx->device) {
            if (p->device >= 0) {
                (void)hipSetDevice(p->device);
                p->release();
            }
            p->device = r1->ctx->device;
        }
        status = hipSetDevice(p->device) == hipSuccess ? PPG_OK : PPG_DEVICE_ERROR;
        s = r1->ctx->stream;
        ppg_shard *sh[2] = {r1, r2};
        for (int f = 0; f < 2 && status == PPG_OK; f++) {
            int64_t n = 0;
            status = local_keys(p, f, sh[f], s, k[f], n);
        }
    }
    int rc;
    if (nranks == 1) rc = status != PPG_OK ? status : check_local(p, k, s);
    else rc = check_dist(p, comm, k, status, s);
    if (rc != PPG_OK) return rc;
    p->checked = true;
    if (result) *result = p->res;
    return PPG_OK;
}

int ppg_pairs_records(const ppg_pairs *p, int32_t file, int64_t lo, int64_t hi, int64_t *shard_record) {
    if (!p || !p->checked || file < 0 || file > 1 || lo < 0 || hi < lo || (hi > lo && !shard_record))
        return PPG_ARG_ERROR;
    const std::vector<int64_t> &dp = p->dp[file];
    for (int64_t i = lo; i < hi; i++) {
        const int64_t d = i - p->start[file];   // this rank's deduplicated number
        if (i >= p->res.pairs || d < 0 || d >= p->local[file]) {
            shard_record[i - lo] = -1;
            continue;
        }
        shard_record[i - lo] = d + (int64_t)(std::upper_bound(dp.begin(), dp.end(), d) - dp.begin());
    }
    return PPG_OK;
}

int ppg_pairs_emit_begin(ppg_pairs *p, ppg_shard *r1, ppg_shard *r2, ppg_comm *comm, int64_t pair_chunk,
                         int64_t window_bytes) {
    if (!p || !p->checked || !r1 || !r2 || pair_chunk < 1) return PPG_ARG_ERROR;
    int32_t rank = 0, nranks = 1;
    if (comm) comm_size(comm, &rank, &nranks);
    if (nranks != p->nranks || rank != p->rank) return PPG_ARG_ERROR;   // the check's comm
    PairEmit &E = p->em;
    E.on = false;
    E.K = pair_chunk;
    E.npc = (p->res.pairs + pair_chunk - 1) / pair_chunk;
    E.sh[0] = r1;
    E.sh[1] = r2;
    E.comm = comm;
    E.exchanged = false;
    E.next = E.w0 = E.w1 = 0;
    E.window_bytes = window_bytes > 0 ? window_bytes : (int64_t)8 << 30;
    E.clen[0] = E.clen[1] = E.cnrec[0] = E.cnrec[1] = 0;
    E.reruns = 0;
    E.fused = false;
    for (double &t : E.t_ms) t = 0;
    for (int f = 0; f < 2; f++) {
        ppg_shard *sh = E.sh[f];
        if (!sh->ran || sh->last_rc != PPG_OK) return PPG_ARG_ERROR;
        if (nranks > 1 && sh->batches.size() != 1) return PPG_UNSUPPORTED;   // N ranks: resident shards only
        E.offst[f].assign((size_t)sh->n, 0);
        uint64_t o = 0;
        for (int32_t k = 0; k < sh->n; k++) {
            E.offst[f][(size_t)k] = o;
            o += sh->h_jobs[(size_t)k].raw_shift;
        }
        E.kvalid[f] = sh->n;
        E.pos[f].resize(p->dp[f].size());
        for (size_t t = 0; t < p->dp[f].size(); t++) E.pos[f][t] = p->dp[f][t] + (int64_t)t;
        // each batch's deduplicated record range
        E.blo[f].clear();
        E.bhi[f].clear();
        for (auto [b0, b1] : sh->batches) {
            const int64_t r0 = sh->h_base[(size_t)b0], r1e = b1 < sh->n ? sh->h_base[(size_t)b1] : sh->total_records;
            E.blo[f].push_back(dedup_of(E.pos[f], r0));
            E.bhi[f].push_back(dedup_of(E.pos[f], r1e));
        }
        E.batch[f] = (int32_t)sh->batches.size() - 1;   // what the run left resident
    }
    if (nranks == 1) {
        E.j_lo = 0;
        E.j_hi = E.npc;
        // the windows' deduplicated numbering is this rank's: pairs beyond either file's records do not exist
        for (int f = 0; f < 2; f++)
            if (E.bhi[f].empty() ? p->res.pairs > 0 : E.bhi[f].back() < p->res.pairs) return PPG_ARG_ERROR;
        if (pairs_perturb() == 1)
            for (int f = 0; f < 2; f++) E.bhi[f].back() = std::max(E.blo[f].back(), E.bhi[f].back() - E.K);
    } else {
        if (p->st[0].size() != (size_t)nranks + 1 || p->st[1].size() != (size_t)nranks + 1) return PPG_ARG_ERROR;
        E.j_lo = E.j_hi = 0;   // set by the exchange
    }
    E.on = true;
    return PPG_OK;
}

int ppg_pairs_emit_run(ppg_pairs *p, ppg_shard *r1, ppg_shard *r2, int64_t pair_chunk, int64_t window_bytes) {
    if (!p || !r1 || !r2 || pair_chunk < 1 || r1 == r2 || r1->ctx->device != r2->ctx->device) return PPG_ARG_ERROR;
    if (!r1->keys_dev || !r2->keys_dev) return PPG_ARG_ERROR;   // the numbering needs each batch's spot keys
    if (p->device != r1->ctx->device) {
        if (p->device >= 0) {
            (void)hipSetDevice(p->device);
            p->release();
        }
        p->device = r1->ctx->device;
    }
    HIPCHK(hipSetDevice(p->device));
    p->checked = false;
    p->res = ppg_pair_result{};
    p->rank = 0;
    p->nranks = 1;
    p->start[0] = p->start[1] = 0;
    PairEmit &E = p->em;
    E.on = false;
    E.fused = true;
    E.K = pair_chunk;
    E.npc = INT64_MAX;   // known once both files have run
    E.sh[0] = r1;
    E.sh[1] = r2;
    E.comm = nullptr;
    E.exchanged = false;
    E.next = E.w0 = E.w1 = 0;
    E.window_bytes = window_bytes > 0 ? window_bytes : (int64_t)8 << 30;
    E.reruns = 0;
    for (double &t : E.t_ms) t = 0;
    E.j_lo = 0;
    E.j_hi = INT64_MAX;
    for (int f = 0; f < 2; f++) {
        ppg_shard *sh = E.sh[f];
        shard_reset(sh);
        sh->keys_written = 0;
        sh->last_rc = PPG_OK;
        E.clen[f] = E.cnrec[f] = 0;
        E.done[f] = false;
        E.run_ms[f] = 0;
        E.batch[f] = -1;
        E.kvalid[f] = 0;
        E.blo[f].clear();
        E.bhi[f].clear();
        E.pos[f].clear();
        p->dp[f].clear();
        p->local[f] = 0;
        E.offst[f].assign((size_t)sh->n, 0);
        uint64_t o = 0;
        for (int32_t k = 0; k < sh->n; k++) {
            E.offst[f][(size_t)k] = o;
            o += sh->h_jobs[(size_t)k].raw_shift;
        }
    }
    E.on = true;
    return PPG_OK;
}

int ppg_pairs_emit_next(ppg_pairs *p, int64_t *j0, int64_t *j1) {
    if (!p || !p->em.on) return PPG_ARG_ERROR;
    HIPCHK(hipSetDevice(p->device));
    PairEmit &E = p->em;
    if (E.fused) {
        const int rc = emit_next_fused(p, j0, j1);
        if (rc < 0) E.on = false;
        return rc;
    }
    if (p->nranks > 1) {
        if (E.exchanged) return PPG_STREAM_END;
        const int rc = emit_exchange(p, j0, j1);
        if (rc != PPG_OK) { E.on = false; return rc; }
        return E.w0 < E.w1 ? PPG_OK : PPG_STREAM_END;
    }
    const int rc = emit_next_local(p, j0, j1);
    if (rc < 0) E.on = false;
    return rc;
}

int ppg_pairs_chunk(ppg_pairs *p, int64_t j, int32_t file, const uint8_t **bytes, int64_t *len, const uint32_t **desc,
                    int64_t *nrec) {
    if (!p || !p->em.on || file < 0 || file > 1 || j < p->em.w0 || j >= p->em.w1) return PPG_ARG_ERROR;
    const PairEmit &E = p->em;
    const size_t i = (size_t)(j - E.w0);
    if (bytes) *bytes = E.bytes[file].p + E.boff[file][i];
    if (len) *len = E.blen[file][i];
    if (desc) *desc = E.desc[file].p + 4 * E.roff[file][i];
    if (nrec) *nrec = E.rcnt[file][i];
    return PPG_OK;
}

int ppg_pairs_copy_chunk(ppg_pairs *p, int64_t j, int32_t file, uint8_t *dst, int64_t cap, int64_t *len, uint32_t *desc,
                         int64_t desc_cap, int64_t *nrec) {
    const uint8_t *b = nullptr;
    const uint32_t *d = nullptr;
    int64_t n = 0, r = 0;
    if (int rc = ppg_pairs_chunk(p, j, file, &b, &n, &d, &r)) return rc;
    if (len) *len = n;
    if (nrec) *nrec = r;
    if ((dst && n > cap) || (desc && r > desc_cap)) return PPG_BUF_ERROR;
    HIPCHK(hipSetDevice(p->device));
    if (dst && n) HIPCHK(hipMemcpy(dst, b, (size_t)n, hipMemcpyDeviceToHost));
    if (desc && r) HIPCHK(hipMemcpy(desc, d, 16 * (size_t)r, hipMemcpyDeviceToHost));
    return PPG_OK;
}

int ppg_pairs_emit_stats(const ppg_pairs *p, double *vals, int32_t n) {
    if (!p || !vals || n < 0) return PPG_ARG_ERROR;
    const PairEmit &E = p->em;
    const double v[8] = {E.t_ms[0], E.t_ms[1], E.t_ms[2], E.t_ms[3], (double)E.reruns, (double)E.npc, (double)E.j_lo,
                         (double)E.j_hi};
    for (int32_t i = 0; i < n && i < 8; i++) vals[i] = v[i];
    return PPG_OK;
}

}  // extern "C"

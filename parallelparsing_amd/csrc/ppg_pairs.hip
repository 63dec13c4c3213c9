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

hipError_t ppg_launch_record_keys(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  const PpgParseInfo *info, const uint64_t *base, const uint32_t *recs, int64_t *keys,
                                  int n);

struct ppg_pairs {
    int device = -1;
    int32_t rank = 0, nranks = 1;
    int64_t local[2] = {0, 0}, start[2] = {0, 0};   // deduplicated records of this rank / before it
    std::vector<int64_t> dp[2];                     // D[t] - t of the sorted duplicate positions
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

}  // extern "C"

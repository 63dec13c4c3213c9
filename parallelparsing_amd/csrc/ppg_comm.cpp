// ppg_comm.cpp — multi-GPU DecompressAll inside the C ABI (include/ppgpu.h, "multi-GPU").
//
// The reference fans DecompressAll out over threads of one host (BatchedFASTQ.cs:62-77: a task per
// chunk pulled from LazyFileReader, records pushed into one RecordCache).  Here the fan-out is
// over GPUs, one process (or host thread) per GPU: rank r decodes a contiguous range of chunks
// balanced by compressed bytes (ppg_partition), with no data-path exchange, and the one collective
// is an all-gather of per-chunk record counts followed by an exclusive scan, which gives every
// chunk its global record number.  RCCL has no all-gatherv: counts are padded to the
// widest range and gathered with ncclAllGather over xGMI on the ctx stream.
//
// Transports of a ppg_comm:
//   RCCL      ppg_comm_init (a communicator of our own from a unique id the host distributes) or
//             ppg_comm_from_rccl (a caller's ncclComm_t).  librccl is dlopen'ed, so a process that
//             already holds one (torch bundles its own librccl.so.1) shares it.
//   host      ppg_comm_init_host: POSIX shared memory between processes of one machine.  RCCL
//             refuses two ranks on one GPU ("Duplicate GPU detected"), so this is how the N > 1
//             path is rehearsed on a one-GPU box; the gather code above it is the same.
#include "ppg_host.h"
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>

namespace {

struct Rccl {
    void *h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char *(*err)(ncclResult_t) = nullptr;
    ncclResult_t (*version)(int *) = nullptr;
    // point-to-point (the paired-read key exchange, ppg_pairs.hip); optional
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    bool load() {
        if (h) return true;
        // the copy already in the process (torch's), else the ROCm one
        for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) return false;
        get_unique_id = (decltype(get_unique_id))dlsym(h, "ncclGetUniqueId");
        init_rank = (decltype(init_rank))dlsym(h, "ncclCommInitRank");
        all_gather = (decltype(all_gather))dlsym(h, "ncclAllGather");
        destroy = (decltype(destroy))dlsym(h, "ncclCommDestroy");
        err = (decltype(err))dlsym(h, "ncclGetErrorString");
        version = (decltype(version))dlsym(h, "ncclGetVersion");
        send = (decltype(send))dlsym(h, "ncclSend");
        recv = (decltype(recv))dlsym(h, "ncclRecv");
        group_start = (decltype(group_start))dlsym(h, "ncclGroupStart");
        group_end = (decltype(group_end))dlsym(h, "ncclGroupEnd");
        return get_unique_id && init_rank && all_gather && destroy && err;
    }
};

Rccl &rccl() {
    static Rccl r;
    return r;
}

#define RCCLCHK(x)                                                                                  \
    do {                                                                                            \
        ncclResult_t r_ = (x);                                                                      \
        if (r_ != ncclSuccess) {                                                                    \
            fprintf(stderr, "ppgpu: %s failed: %s\n", #x, rccl().err ? rccl().err(r_) : "?");       \
            return PPG_DEVICE_ERROR;                                                                \
        }                                                                                           \
    } while (0)

// shared-memory all-gather between the processes of one machine (sense-reversing barrier).  Rank 0
// creates the segment (O_EXCL: a name must be unique per job, a stale segment is never reused),
// zeroes it and publishes magic + nranks last; the other ranks join only after seeing both.  A
// barrier that times out poisons the segment: every later call on it fails instead of miscounting.
struct ShmHdr {
    std::atomic<uint64_t> arrive;
    std::atomic<uint64_t> gen;
    std::atomic<uint64_t> magic;
    std::atomic<uint64_t> nranks;
    std::atomic<uint64_t> poison;
};
static_assert(sizeof(ShmHdr) <= 64, "header fits the segment's first 64 bytes");
constexpr uint64_t kShmMagic = 0x7070677368636F6Dull;   // "ppgshcom"
constexpr int64_t kShmSlot = 8 << 20;   // bytes per rank per all-gather (1M chunk counts)
constexpr int kShmTimeoutS = 300;
constexpr size_t kStatSlots = 64;       // int64 per rank in the buffer made with an RCCL comm (status and per-peer size gathers)

}  // namespace

struct ppg_comm {
    int32_t nranks = 1, rank = 0;
    int device = -1;                    // RCCL: the GPU the communicator was made for
    ncclComm_t nccl = nullptr;
    bool own_nccl = false;
    // RCCL: the gathers run on the communicator's own stream, from buffers it owns; the status
    // phase's buffer is allocated when the comm is made, so nothing can fail before a rank joins it
    hipStream_t stream = nullptr;
    DevBuf<int64_t> stat;               // [0] = this rank's (status, width), [2..] = every rank's
    DevBuf<int64_t> data;               // the padded counts (grown between the two phases)
    // host transport
    std::string shm_name;
    ShmHdr *hdr = nullptr;
    uint8_t *slots = nullptr;
    size_t map_len = 0;
    bool poisoned = false;

    bool host() const { return hdr != nullptr; }

    int barrier() {
        if (poisoned || hdr->poison.load(std::memory_order_acquire)) return PPG_IO_ERROR;
        const uint64_t g = hdr->gen.load(std::memory_order_acquire);
        if (hdr->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint64_t)nranks) {
            hdr->arrive.store(0, std::memory_order_relaxed);
            hdr->gen.store(g + 1, std::memory_order_release);
            return PPG_OK;
        }
        const auto t0 = std::chrono::steady_clock::now();
        while (hdr->gen.load(std::memory_order_acquire) == g) {
            std::this_thread::yield();
            if (hdr->poison.load(std::memory_order_acquire)) { poisoned = true; return PPG_IO_ERROR; }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(kShmTimeoutS)) {
                // the arrive count is now wrong for every later barrier: the comm is dead
                poisoned = true;
                hdr->poison.store(1, std::memory_order_release);
                return PPG_IO_ERROR;
            }
        }
        return PPG_OK;
    }

    // host memory in, host memory out: recv = nranks * bytes
    int host_all_gather(const void *send, void *recv, int64_t bytes) {
        if (bytes > kShmSlot) return PPG_UNSUPPORTED;
        memcpy(slots + (size_t)rank * kShmSlot, send, (size_t)bytes);
        if (int rc = barrier()) return rc;
        for (int32_t r = 0; r < nranks; r++) memcpy((uint8_t *)recv + (size_t)r * bytes, slots + (size_t)r * kShmSlot,
                                                    (size_t)bytes);
        return barrier();   // nobody overwrites a slot before every rank has read it
    }

    // RCCL all-gather of n int64 per rank: send = buf[0, n), recv = buf[n, n + n * nranks), on
    // the comm's stream; host copies in and out.  A failed copy in still enters the collective
    // (with stale data: the others are waiting) and is reported through sent_ok; an error return
    // means the collective itself failed.
    int rccl_all_gather(DevBuf<int64_t> &buf, const int64_t *send, int64_t *recv, size_t n, bool &sent_ok) {
        sent_ok = hipMemcpyAsync(buf.p, send, 8 * n, hipMemcpyHostToDevice, stream) == hipSuccess;
        RCCLCHK(rccl().all_gather(buf.p, buf.p + n, n, ncclInt64, nccl, stream));
        HIPCHK(hipMemcpyAsync(recv, buf.p + n, 8 * n * (size_t)nranks, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        return PPG_OK;
    }

    // RCCL side state, made with the communicator (on its device)
    int rccl_setup() {
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        HIPCHK(stat.alloc(kStatSlots * ((size_t)nranks + 1)));
        return PPG_OK;
    }
};

extern "C" {

int ppg_comm_unique_id(uint8_t *id) {
    if (!id) return PPG_ARG_ERROR;
    if (!rccl().load()) return PPG_UNSUPPORTED;
    ncclUniqueId u;
    RCCLCHK(rccl().get_unique_id(&u));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return PPG_OK;
}

int ppg_comm_init(ppg_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t *id, ppg_comm **out) {
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return PPG_ARG_ERROR;
    if (!rccl().load()) return PPG_UNSUPPORTED;
    HIPCHK(hipSetDevice(ctx->device));
    auto c = std::make_unique<ppg_comm>();
    c->nranks = nranks;
    c->rank = rank;
    c->device = ctx->device;
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    RCCLCHK(rccl().init_rank(&c->nccl, nranks, u, rank));
    c->own_nccl = true;
    if (int rc = c->rccl_setup()) { ppg_comm_free(c.release()); return rc; }
    *out = c.release();
    return PPG_OK;
}

int ppg_comm_from_rccl(ppg_ctx *ctx, void *nccl_comm, int32_t nranks, int32_t rank, ppg_comm **out) {
    if (!ctx || !nccl_comm || !out || nranks < 1 || rank < 0 || rank >= nranks) return PPG_ARG_ERROR;
    if (!rccl().load()) return PPG_UNSUPPORTED;
    auto c = std::make_unique<ppg_comm>();
    c->nranks = nranks;
    c->rank = rank;
    c->device = ctx->device;
    c->nccl = (ncclComm_t)nccl_comm;
    if (int rc = c->rccl_setup()) { ppg_comm_free(c.release()); return rc; }
    *out = c.release();
    return PPG_OK;
}

int ppg_comm_init_host(int32_t nranks, int32_t rank, const char *name, ppg_comm **out) {
    if (!name || !out || nranks < 1 || rank < 0 || rank >= nranks || name[0] != '/') return PPG_ARG_ERROR;
    auto c = std::make_unique<ppg_comm>();
    c->nranks = nranks;
    c->rank = rank;
    c->shm_name = name;
    c->map_len = 64 + (size_t)nranks * kShmSlot;
    const auto t0 = std::chrono::steady_clock::now();
    void *p = MAP_FAILED;
    if (rank == 0) {
        // a fresh segment (zero-filled by ftruncate); an existing name is an error, never reused
        const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) return PPG_IO_ERROR;
        if (ftruncate(fd, (off_t)c->map_len) == 0)
            p = mmap(nullptr, c->map_len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) { shm_unlink(name); return PPG_IO_ERROR; }
        c->hdr = (ShmHdr *)p;
        c->hdr->nranks.store((uint64_t)nranks, std::memory_order_relaxed);
        c->hdr->magic.store(kShmMagic, std::memory_order_release);   // published last
    } else {
        // wait for rank 0's segment: it exists, has its full size and carries magic + nranks
        for (;;) {
            const int fd = shm_open(name, O_RDWR, 0600);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && (size_t)st.st_size >= c->map_len)
                    p = mmap(nullptr, c->map_len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                close(fd);
                if (p != MAP_FAILED) {
                    ShmHdr *h = (ShmHdr *)p;
                    if (h->magic.load(std::memory_order_acquire) == kShmMagic) {
                        if (h->nranks.load(std::memory_order_relaxed) != (uint64_t)nranks) {
                            munmap(p, c->map_len);
                            return PPG_ARG_ERROR;
                        }
                        break;
                    }
                    munmap(p, c->map_len);
                    p = MAP_FAILED;
                }
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(kShmTimeoutS)) return PPG_IO_ERROR;
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        c->hdr = (ShmHdr *)p;
    }
    c->slots = (uint8_t *)p + 64;
    // every rank has mapped the segment before any gather starts
    if (int rc = c->barrier()) {
        munmap(p, c->map_len);
        if (rank == 0) shm_unlink(name);
        return rc;
    }
    *out = c.release();
    return PPG_OK;
}

void ppg_comm_free(ppg_comm *c) {
    if (!c) return;
    if (c->nccl) {
        if (c->device >= 0) (void)hipSetDevice(c->device);
        if (c->own_nccl) (void)rccl().destroy(c->nccl);
        c->stat.release();
        c->data.release();
        if (c->stream) (void)hipStreamDestroy(c->stream);
    }
    if (c->hdr) {
        munmap((void *)c->hdr, c->map_len);
        if (c->rank == 0) shm_unlink(c->shm_name.c_str());
    }
    delete c;
}

int ppg_comm_rank(const ppg_comm *c, int32_t *rank, int32_t *nranks) {
    if (!c) return PPG_ARG_ERROR;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return PPG_OK;
}

int ppg_rccl_version(int *version) {
    if (!version) return PPG_ARG_ERROR;
    if (!rccl().load() || !rccl().version) return PPG_UNSUPPORTED;
    RCCLCHK(rccl().version(version));
    return PPG_OK;
}

// Contiguous chunk ranges balanced by compressed bytes (chunk k reads Input[k+1] - Input[k] + 1
// bytes, LazyFileReader.cs:64): rank r owns chunks [bounds[r], bounds[r+1]) of [first, first+n).
int ppg_partition(const ppg_index *ix, int32_t first, int32_t n, int32_t nranks, int32_t *bounds) {
    if (!ix || !bounds || nranks < 1 || first < 0 || n < 0 || (size_t)first + (size_t)n + 1 > ix->pts.size())
        return PPG_ARG_ERROR;
    const auto &P = ix->pts;
    std::vector<double> cum((size_t)n + 1, 0.0);
    for (int32_t k = 0; k < n; k++)
        cum[(size_t)k + 1] = cum[(size_t)k] + (double)(P[(size_t)first + k + 1].input - P[(size_t)first + k].input + 1);
    bounds[0] = first;
    for (int32_t r = 1; r < nranks; r++) {
        const double target = cum[(size_t)n] * r / nranks;
        int32_t k = (int32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        k = std::min(std::max(k, bounds[r - 1] - first), n);
        bounds[r] = first + k;
    }
    bounds[nranks] = first + n;
    return PPG_OK;
}

}  // extern "C"

// The count all-gather, in two phases that every rank always enters, failed or not (a rank that
// returned early would leave the others waiting in the collective forever):
//   1. (status, width) of every rank, from a buffer allocated with the comm -- a failing rank,
//      one whose bounds are bad or whose data buffer cannot be allocated says so here;
//   2. only if every rank is fine (each rank decides from the same gathered statuses): the
//      per-chunk counts padded to the widest range (RCCL has no all-gatherv).
// Every rank returns the first failing rank's status.  bounds may be NULL (a rank that could not
// partition); ctx may be NULL (a host-transport comm, or a failed rank).
static int gather_counts(ppg_comm *comm, ppg_ctx *ctx, const std::vector<int64_t> &local, int status,
                         const int32_t *bounds, int64_t *counts, int64_t *bases, int64_t *total_records) {
    const int32_t R = comm->nranks;
    int32_t width = 1;
    if (!bounds) {
        if (status == PPG_OK) status = PPG_ARG_ERROR;
    } else {
        for (int32_t r = 0; r < R; r++) {
            if (bounds[r + 1] < bounds[r]) { if (status == PPG_OK) status = PPG_ARG_ERROR; width = 1; break; }
            width = std::max(width, bounds[r + 1] - bounds[r]);
        }
        if (status == PPG_OK && (int64_t)local.size() != bounds[comm->rank + 1] - bounds[comm->rank])
            status = PPG_ARG_ERROR;
    }
    const int32_t W = width;
    const bool rccl_path = !comm->host();
    if (rccl_path) {
        if (hipSetDevice(comm->device) != hipSuccess && status == PPG_OK) status = PPG_DEVICE_ERROR;
        if (ctx && comm->device != ctx->device && status == PPG_OK) status = PPG_ARG_ERROR;
        if (status == PPG_OK && comm->data.alloc((size_t)W * (R + 1)) != hipSuccess) status = PPG_MEM_ERROR;
    } else if (8 * (int64_t)W > kShmSlot && status == PPG_OK) {
        status = PPG_UNSUPPORTED;
    }
    // phase 1: statuses and widths
    int64_t mine[2] = {status, W};
    std::vector<int64_t> all(2 * (size_t)R, 0);
    bool sent_ok = true;
    // a failed collective (RCCL error, host-transport timeout / poison) is the only early return
    if (int rc1 = rccl_path ? comm->rccl_all_gather(comm->stat, mine, all.data(), 2, sent_ok)
                            : comm->host_all_gather(mine, all.data(), 16))
        return rc1;
    for (int32_t r = 0; r < R; r++)
        if (all[2 * (size_t)r] != 0) return (int)all[2 * (size_t)r];
    for (int32_t r = 0; r < R; r++)
        if (all[2 * (size_t)r + 1] != W) return PPG_ARG_ERROR;   // ranks disagree on the bounds
    if (!sent_ok) status = PPG_DEVICE_ERROR;   // the others saw a stale "ok": gather anyway, then fail
    // phase 2: the counts
    std::vector<int64_t> send((size_t)W, 0), recv((size_t)W * R, 0);
    std::copy(local.begin(), local.end(), send.begin());
    const int rc2 = rccl_path ? comm->rccl_all_gather(comm->data, send.data(), recv.data(), (size_t)W, sent_ok)
                              : comm->host_all_gather(send.data(), recv.data(), 8 * (int64_t)W);
    if (status != PPG_OK) return status;
    if (rc2 != PPG_OK) return rc2;
    if (!sent_ok) return PPG_DEVICE_ERROR;
    int64_t run = 0;
    size_t o = 0;
    for (int32_t r = 0; r < R; r++)
        for (int32_t i = 0; i < bounds[r + 1] - bounds[r]; i++, o++) {
            const int64_t c = recv[(size_t)r * W + i];
            if (counts) counts[o] = c;
            if (bases) bases[o] = run;
            run += c;
        }
    if (total_records) *total_records = run;
    return PPG_OK;
}

extern "C" {

// After ppg_shard_run on every rank (rank r's shard = chunks [bounds[r], bounds[r+1])): one
// all-gather of the per-chunk record counts, padded to the widest range, then the exclusive scan.
// counts / bases (may be NULL) receive bounds[nranks] - bounds[0] entries in canonical order.
int ppg_shard_gather_counts(ppg_shard *sh, ppg_comm *comm, const int32_t *bounds, int64_t *counts, int64_t *bases,
                            int64_t *total_records) {
    if (!comm) return PPG_ARG_ERROR;   // nothing to join
    // from here on every path joins the gather: the other ranks wait for this one
    int status = PPG_OK;
    std::vector<int64_t> local;
    if (!sh) {
        status = PPG_ARG_ERROR;
    } else if (sh->last_rc != PPG_OK) {
        status = sh->last_rc;                          // the rank's own DecompressAll failed
    } else if (!sh->ran || !bounds || bounds[comm->rank + 1] - bounds[comm->rank] != sh->n) {
        status = PPG_ARG_ERROR;
    } else {
        local.resize((size_t)sh->n);
        for (int32_t i = 0; i < sh->n; i++) local[(size_t)i] = (int64_t)sh->h_info[(size_t)i].records;
    }
    const int rc = gather_counts(comm, sh ? sh->ctx : nullptr, local, status, bounds, counts, bases, total_records);
    return status != PPG_OK ? status : rc;
}

// Multi-GPU DecompressAll of a .gz file (BatchedFASTQ over every chunk, fanned out over ranks):
// this rank's chunk range (ppg_partition over the comm), its compressed bytes pread from the file
// into HBM, decoded in batches of out_capacity (0: at once), then the count all-gather.  counts /
// bases (may be NULL) get one entry per chunk of the index in canonical order.
int ppg_dist_decompress_all(ppg_ctx *ctx, ppg_comm *comm, const ppg_index *ix, const char *gz_path,
                            int64_t out_capacity, int64_t *counts, int64_t *bases, int64_t *total_records) {
    if (!comm) return PPG_ARG_ERROR;   // nothing to join
    // from here on every path joins the gather: a failure is everyone's result, never a hang
    int rc = (!ctx || !ix || !gz_path || ix->pts.size() < 1) ? PPG_ARG_ERROR : PPG_OK;
    std::vector<int32_t> bounds((size_t)comm->nranks + 1, 0);
    if (rc == PPG_OK) rc = ppg_partition(ix, 0, (int32_t)ix->pts.size() - 1, comm->nranks, bounds.data());
    std::vector<int64_t> local;
    if (rc == PPG_OK) {
        const int32_t a = bounds[(size_t)comm->rank], b = bounds[(size_t)comm->rank + 1];
        const int fd = open(gz_path, O_RDONLY);
        struct FdClose { int fd; ~FdClose() { if (fd >= 0) close(fd); } } fdc{fd};
        const int64_t lo = ix->pts[(size_t)a].input - 1, len = ix->pts[(size_t)b].input - ix->pts[(size_t)a].input + 1;
        PinnedBuf pin;
        rc = fd < 0 ? PPG_IO_ERROR
             : hipSetDevice(ctx->device) == hipSuccess && pin.alloc((size_t)std::max<int64_t>(len, 1)) == hipSuccess
                 ? PPG_OK : PPG_DEVICE_ERROR;
        if (rc == PPG_OK && len > 0 && !pread_parallel(fd, pin.p, lo, len, 8)) rc = PPG_IO_ERROR;
        ppg_shard *sh = nullptr;
        if (rc == PPG_OK) rc = ppg_shard_create(ctx, ix, a, b - a, pin.p, len, 0, out_capacity, &sh);
        if (rc == PPG_OK) rc = ppg_shard_run(sh);
        if (rc == PPG_OK) {
            local.resize((size_t)(b - a));
            for (int32_t i = 0; i < b - a; i++) local[(size_t)i] = (int64_t)sh->h_info[(size_t)i].records;
        }
        ppg_shard_free(sh);
    }
    const int grc = gather_counts(comm, ctx, local, rc, rc == PPG_OK ? bounds.data() : nullptr, counts, bases,
                                  total_records);
    return rc != PPG_OK ? rc : grc;
}

}  // extern "C"

// ---- collectives for the other multi-rank steps of the library (ppg_pairs.hip) ----

int comm_size(const ppg_comm *c, int32_t *rank, int32_t *nranks) { return ppg_comm_rank(c, rank, nranks); }
int comm_device(const ppg_comm *c) { return c->host() ? -1 : c->device; }

// All-gather of n <= 64 int64 per rank (statuses, counts, per-peer sizes), host memory in and out, over either
// transport, from a buffer made with the comm (nothing to allocate, so every rank always joins).
// sent_ok reports a failed copy into the collective (the others then got stale data).
int comm_all_gather_i64(ppg_comm *c, const int64_t *send, int64_t *recv, size_t n, bool &sent_ok) {
    sent_ok = true;
    if (c->host()) return c->host_all_gather(send, recv, 8 * (int64_t)n);
    if (n > kStatSlots) return PPG_UNSUPPORTED;   // status-sized gathers only: the buffer exists already
    HIPCHK(hipSetDevice(c->device));
    return c->rccl_all_gather(c->stat, send, recv, n, sent_ok);
}

// All-to-all-v of int64 between device buffers on this rank's GPU.  m = the R x R count matrix
// (m[src * R + dst] elements), known to every rank; send / recv are laid out by destination /
// source in rank order.  RCCL: grouped ncclSend / ncclRecv on the comm's stream (xGMI
// point-to-point); host transport: staged through host memory in rounds of the shared slots.
// The caller's stream s must have produced `send` (it is synchronised first).  Every rank runs
// every round whatever its own errors (the others would wait); the first error is returned after.
// The grouped ncclSend / ncclRecv of one all-to-all-v, with the group ALWAYS closed: a send or recv
// that fails to enqueue stops further enqueues, but ncclGroupEnd still runs, so this rank neither
// leaves a group open on its thread (the next collective on the comm would misbehave instead of
// failing) nor returns before the group's launch.  The first error is returned.  The
// RCCL entry points come in as a table so host_check can drive the error paths without a GPU.
int comm_grouped_p2p(const CommP2P &f, void *comm, hipStream_t stream, const int64_t *send, int64_t *recv,
                     const int64_t *m, int32_t R, int32_t me, const int64_t *sd, const int64_t *rd) {
    ncclResult_t first = f.group_start();
    if (first != ncclSuccess) {
        fprintf(stderr, "ppgpu: ncclGroupStart failed: %s\n", f.err ? f.err(first) : "?");
        return PPG_DEVICE_ERROR;   // no group was opened
    }
    const char *what = nullptr;
    for (int32_t q = 0; q < R && first == ncclSuccess; q++) {
        if (q == me) continue;
        if (m[(size_t)me * R + q]) {
            first = f.send(send + sd[q], (size_t)m[(size_t)me * R + q], ncclInt64, q, (ncclComm_t)comm, stream);
            what = "ncclSend";
        }
        if (first == ncclSuccess && m[(size_t)q * R + me]) {
            first = f.recv(recv + rd[q], (size_t)m[(size_t)q * R + me], ncclInt64, q, (ncclComm_t)comm, stream);
            what = "ncclRecv";
        }
    }
    const ncclResult_t end = f.group_end();
    if (first != ncclSuccess) {
        fprintf(stderr, "ppgpu: %s failed: %s\n", what, f.err ? f.err(first) : "?");
        return PPG_DEVICE_ERROR;
    }
    if (end != ncclSuccess) {
        fprintf(stderr, "ppgpu: ncclGroupEnd failed: %s\n", f.err ? f.err(end) : "?");
        return PPG_DEVICE_ERROR;
    }
    return PPG_OK;
}

int comm_alltoallv_i64(ppg_comm *c, hipStream_t s, const int64_t *send, int64_t *recv, const int64_t *m,
                       bool on_device) {
    const int32_t R = c->nranks, me = c->rank;
    std::vector<int64_t> sd((size_t)R + 1, 0), rd((size_t)R + 1, 0);
    for (int32_t q = 0; q < R; q++) {
        sd[(size_t)q + 1] = sd[(size_t)q] + m[(size_t)me * R + q];
        rd[(size_t)q + 1] = rd[(size_t)q] + m[(size_t)q * R + me];
    }
    int rc = !s || hipStreamSynchronize(s) == hipSuccess ? PPG_OK : PPG_DEVICE_ERROR;
    if (!c->host()) {
        if (!on_device) return PPG_ARG_ERROR;   // RCCL moves device memory only
        if (!rccl().send || !rccl().recv || !rccl().group_start || !rccl().group_end) return PPG_UNSUPPORTED;
        HIPCHK(hipSetDevice(c->device));
        const CommP2P f{rccl().send, rccl().recv, rccl().group_start, rccl().group_end, rccl().err};
        if (int g = comm_grouped_p2p(f, c->nccl, c->stream, send, recv, m, R, me, sd.data(), rd.data())) return g;
        if (m[(size_t)me * R + me])
            HIPCHK(hipMemcpyAsync(recv + rd[(size_t)me], send + sd[(size_t)me], 8 * (size_t)m[(size_t)me * R + me],
                                  hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return rc;
    }
    // host transport: this rank's outgoing keys to host memory, rounds through the slots, back
    std::vector<int64_t> hs, hr;
    const int64_t *src_all = send;
    int64_t *dst_all = recv;
    if (on_device) {
        hs.resize((size_t)sd[(size_t)R]);
        hr.resize((size_t)rd[(size_t)R]);
        if (rc == PPG_OK && !hs.empty() && hipMemcpy(hs.data(), send, 8 * hs.size(), hipMemcpyDeviceToHost) != hipSuccess)
            rc = PPG_DEVICE_ERROR;
        src_all = hs.data();
        dst_all = hr.data();
    }
    const int64_t quota = kShmSlot / 8 / R;   // elements per (src, dst) per round
    int64_t maxc = 0;
    for (int64_t i = 0; i < (int64_t)R * R; i++) maxc = std::max(maxc, m[i]);
    const int64_t rounds = (maxc + quota - 1) / quota;
    for (int64_t t = 0; t < rounds; t++) {
        int64_t *mine = (int64_t *)(c->slots + (size_t)me * kShmSlot);
        for (int32_t q = 0; q < R; q++) {
            const int64_t n = std::min(quota, std::max<int64_t>(0, m[(size_t)me * R + q] - t * quota));
            if (n) memcpy(mine + (size_t)q * quota, src_all + sd[(size_t)q] + t * quota, 8 * (size_t)n);
        }
        if (int b = c->barrier()) return b;
        for (int32_t q = 0; q < R; q++) {
            const int64_t n = std::min(quota, std::max<int64_t>(0, m[(size_t)q * R + me] - t * quota));
            const int64_t *src = (const int64_t *)(c->slots + (size_t)q * kShmSlot) + (size_t)me * quota;
            if (n) memcpy(dst_all + rd[(size_t)q] + t * quota, src, 8 * (size_t)n);
        }
        if (int b = c->barrier()) return b;
    }
    if (on_device && rc == PPG_OK && !hr.empty() &&
        hipMemcpy(recv, hr.data(), 8 * hr.size(), hipMemcpyHostToDevice) != hipSuccess)
        rc = PPG_DEVICE_ERROR;
    return rc;
}

extern "C" int ppg_comm_alltoallv(ppg_comm *c, const int64_t *send, int64_t *recv, const int64_t *counts,
                                  int on_device) {
    if (!c || !counts) return PPG_ARG_ERROR;
    return comm_alltoallv_i64(c, nullptr, send, recv, counts, on_device != 0);
}

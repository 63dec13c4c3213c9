/*
 * ppgpu.h — C ABI of libppgpu.so, the MI355X (gfx950) replacement for the native layer under
 * Quantumzhao/ParallelParsing's chunked-gzip DecompressAll path.
 *
 * The reference reaches native code only through Interop/PlatformInterop.cs:6-35
 * ([DllImport("libz")] inflateInit2_/inflatePrime/inflateSetDictionary/inflate/inflateEnd/
 * inflateReset, driven by Decompressor/Core.cs).  This ABI replaces that layer one level up:
 * a C# host keeps Core/IndexIO/BatchedFASTQ's API surface and binds these entry points with a
 * [DllImport("ppgpu")] class of the same shape as LibZ (INTEGRATION.md shows the stub).
 *
 * Conventions (mirroring Interop/Conventions.cs):
 *  - every entry point returns an int status: PPG_OK (0) or a negative code; the ZResult values
 *    (Conventions.cs:9-20) keep their meaning, device failures get their own codes;
 *  - no exceptions cross the ABI; caller-owned buffers are pinned by the caller (as Core.cs:162,
 *    171 pins Memory<byte>) and never retained; library-owned objects have explicit _free/_close;
 *  - one ppg_ctx per GPU; a ctx is used by one host thread at a time (the reference's
 *    per-call ZStream, Core.cs:136, is likewise single-threaded) -- except ppg_decompress_chunk,
 *    the README's thread-safe "Decompress", which any number of threads may call on one ctx at
 *    once (alongside the one thread using the ctx's other entry points).
 */
#ifndef PPGPU_H
#define PPGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: ZResult (Interop/Conventions.cs:9-20) + library codes ---- */
#define PPG_OK 0
#define PPG_STREAM_END 1
#define PPG_NEED_DICT 2
#define PPG_ERRNO (-1)
#define PPG_STREAM_ERROR (-2)
#define PPG_DATA_ERROR (-3)
#define PPG_MEM_ERROR (-4)
#define PPG_BUF_ERROR (-5)
#define PPG_VERSION_ERROR (-6)
#define PPG_INDEX_OUT_OF_RANGE (-50) /* C# IndexOutOfRangeException (>32 KiB without '@') */
#define PPG_IO_ERROR (-51)
#define PPG_ARG_ERROR (-52)
#define PPG_UNSUPPORTED (-53)        /* input the GPU CreateIndex does not take (not single-member gzip) */
#define PPG_DEVICE_ERROR (-100)
#define PPG_NO_DEVICE (-101)

#define PPG_WINSIZE 32768 /* Common/Constants.cs:9  */
#define PPG_CHUNK 16384   /* Common/Constants.cs:12 */

/* ======================= Index (Common/Index.cs, Common/IndexIO.cs) ======================= */
typedef struct ppg_ctx ppg_ctx;       /* one GPU (see "device context" below) */
typedef struct ppg_index ppg_index;

/* CreateIndex: Core.BuildDeflateIndex(FileStream, uint chunksize) — Decompressor/Core.cs:14-131.
 * Host-side (serial zlib pass, as in the reference).  _mem takes the whole .gz in memory. */
int ppg_index_build_file(const char *gz_path, uint32_t chunksize, ppg_index **out);
int ppg_index_build_mem(const uint8_t *gz, int64_t gz_len, uint32_t chunksize, ppg_index **out);

/* CreateIndex on the GPU: the same Points as ppg_index_build_* (Core.BuildDeflateIndex,
 * Decompressor/Core.cs:14-131) from a block-parallel decode (ppg_index_gpu.cpp): candidate block
 * headers per piece of piece_bytes (0: automatic), a verified chain of block ends, exact output
 * per piece, then the '@' census.  gz: the whole single-member .gz, in host memory or (gz_on_device,
 * 4-byte aligned) in device memory.  out_capacity bounds the exact-output buffer (0: 96 GiB or free HBM less 4 GiB,
 * whichever is smaller; larger members are decoded in batches).
 * Returns PPG_UNSUPPORTED for zlib-wrapped / multi-member input (use ppg_index_build_file). */
int ppg_index_build_gpu(ppg_ctx *ctx, const void *gz, int64_t gz_len, int gz_on_device, uint32_t chunksize,
                        int64_t piece_bytes, int64_t out_capacity, ppg_index **out);

/* ppg_index_build_gpu that also records side points for ppg_shard_set_split: at every block end
 * at least side_bytes of output past the previous Point or side point (and not itself a Point),
 * its absolute bit, output offset and 32 KiB window, gathered on the GPU while the batch's output
 * is resident.  side_bytes <= 0: none.  Side points are not part of the .gzi (IndexIO). */
int ppg_index_build_gpu_side(ppg_ctx *ctx, const void *gz, int64_t gz_len, int gz_on_device, uint32_t chunksize,
                             int64_t piece_bytes, int64_t out_capacity, int64_t side_bytes, ppg_index **out);
int ppg_index_side_count(const ppg_index *ix);
/* copies the side points (any pointer may be NULL): count entries, windows count * 32768 bytes */
int ppg_index_side_points(const ppg_index *ix, int64_t *bit, int64_t *output, uint8_t *windows);
/* replaces the index's side points (a host that found inner block starts itself); sorted by output
 * and bit.  ppg_decompress_chunk splits every chunk at them (ppg_file_decompress_all and ppg_cursor
 * when a piece or batch is too small to fill the GPU). */
int ppg_index_set_side_points(ppg_index *ix, int32_t n, const int64_t *bit, const int64_t *output,
                              const uint8_t *windows);

int ppg_index_build_gpu_file(ppg_ctx *ctx, const char *gz_path, uint32_t chunksize, int64_t piece_bytes,
                             ppg_index **out);
/* Last GPU CreateIndex on ctx: [0] finder ms, [1] pass-1 ms, [2] chain check ms, [3] pass-2 ms,
 * [4] census + windows ms, [5] total ms, [6] pieces, [7] real pieces, [8] pass-1 redos,
 * [9] history resolve ms, [10] pass-2 batches, [11] blocks, [12] points, [13] output bytes,
 * [14] file upload ms (ppg_index_build_gpu_file), [15] pass-2 buffer allocation ms,
 * [16] speculative redos (false starts decoded again from their predecessor's end, one launch),
 * [17] serial redos (false starts the speculation missed).  n <= 18 values are written. */
int ppg_index_build_gpu_stats(ppg_ctx *ctx, double *vals, int32_t n);

/* Serialize / Deserialize — Common/IndexIO.cs:7-27 / :29-53 (byte-identical .gzi format). */
int ppg_index_serialize(const ppg_index *ix, const char *path);
int ppg_index_deserialize(const char *path, ppg_index **out);

/* Build an Index from caller arrays (the form a C# host holding an Index would pass; Point
 * fields of Common/Index.cs:51-82).  windows: count*32768 bytes; offsets concatenated with
 * offset_len[i] bytes each. */
int ppg_index_from_points(int32_t count, const int64_t *output, const int64_t *input, const int32_t *bits,
                          const uint8_t *windows, const int32_t *offset_len, const uint8_t *offsets,
                          int32_t chunk_max_bytes, ppg_index **out);

int32_t ppg_index_count(const ppg_index *ix);                 /* Index.Count (Index.cs:21) */
int32_t ppg_index_chunk_max_bytes(const ppg_index *ix);       /* Index.ChunkMaxBytes (Index.cs:10) */
int ppg_index_point(const ppg_index *ix, int32_t i, int64_t *output, int64_t *input, int32_t *bits,
                    int32_t *offset_len);                     /* Index[i] (Index.cs:20) */
const uint8_t *ppg_index_window(const ppg_index *ix, int32_t i);  /* Point.Window */
const uint8_t *ppg_index_offset(const ppg_index *ix, int32_t i);  /* Point.offset */
void ppg_index_free(ppg_index *ix);

/* Whether chunks [first, first+n) fit the decode kernels (checked by ppg_shard_create and every
 * decode entry point): PPG_OK; PPG_UNSUPPORTED for a chunk whose output (+ its offset carry) is
 * 2^31 bytes or more -- where the reference's (int)(to.Output - from.Output) (Core.cs:140) already
 * breaks -- or whose compressed span is 2^32 - 2^12 bits or more; PPG_ARG_ERROR for Points out of
 * order or a range outside the index.  Host-only; needs no device. */
int ppg_index_validate(const ppg_index *ix, int32_t first, int32_t n);

/* ================================= device context ================================= */

int ppg_device_count(int *n);
int ppg_open(int device, ppg_ctx **out);
void ppg_close(ppg_ctx *ctx);
void *ppg_ctx_stream(ppg_ctx *ctx); /* the hipStream_t every kernel of this ctx runs on */

/* Stream-ordered handoff between the ctx's stream and a caller's hipStream_t (torch's current
 * stream, a host's own), with no host synchronisation -- the device-side counterpart of the
 * reference's per-call ZStream ownership (Interop/Conventions.cs:43-127):
 *   ppg_ctx_wait_stream: work queued on the ctx from now on waits for everything already queued on
 *     `stream` (call it before a ppg call reads device memory that `stream` writes, or writes
 *     memory that `stream` may still read, e.g. a block a caching allocator recycled);
 *   ppg_stream_wait_ctx: work queued on `stream` from now on waits for everything already queued
 *     on the ctx.
 * Every ppg entry point that reads caller device memory (comp_on_device, gz_on_device) or writes it
 * (ppg_shard_keys, ppg_shard_counts_to_device, ppg_shard_copy_output) does so on the ctx's
 * stream, so one ppg_ctx_wait_stream before the call orders it after the caller's producers. */
int ppg_ctx_wait_stream(ppg_ctx *ctx, void *stream);
int ppg_stream_wait_ctx(ppg_ctx *ctx, void *stream);

/* ====================== Decompress one checkpoint (README "Decompress") ======================
 * Core.ExtractDeflateIndex(fileBuffer, from=Index[k], to=Index[k+1], buf) — Core.cs:133-192,
 * plus Parsing.Parse of offset_k ++ chunk (BatchedFASTQ.cs:67-68).  `slice` holds file bytes
 * [Index[k].Input-1, Index[k+1].Input-1] exactly as LazyFileReader reads them
 * (LazyFileReader.cs:63-69).  out receives to.Output-from.Output bytes; `produced` the count
 * (Core.cs:191).  If recs is non-NULL, up to rec_cap records are written as 4 uint32 newline
 * positions (n1..n4) relative to raw = offset_k ++ out; *nrec gets the record count.
 * Thread safe (README.md:38-50): concurrent calls on one ctx are combined into shared launches (four
 * launch slots, each with its own stream and buffers that only grow: no hipMalloc/hipFree per call
 * once warm; a second launch starts beside a decoding one only once 16 calls queue, so the queue
 * that builds up during a launch goes into the next one); every call gets its own chunk's results.
 * A chunk of an index with side points
 * (ppg_index_build_gpu_side) is decoded as one wave per piece; in a launch of at most 4,096 chunks,
 * a chunk of an index without them gets its inner block starts found on the GPU first (candidate
 * block headers, a speculative symbolic decode, the verified chain of block ends from the chunk's
 * Point and their resolved 32 KiB histories -- CreateIndex's own kernels) and is decoded as up to
 * 16 pieces too; in a launch of at most 256 such chunks the search's symbolic decode covers each
 * whole chunk and a chunk whose chain is verified end to end is written out from its symbols, with
 * no second decode.  Environment PPG_CHUNK_NO_FIND=1 turns the search off (PPG_CHUNK_NO_MAT=1 only
 * the write-out from symbols). */
int ppg_decompress_chunk(ppg_ctx *ctx, const ppg_index *ix, int32_t k, const uint8_t *slice, int64_t slice_len,
                         uint8_t *out, int64_t out_cap, int64_t *produced, uint32_t *recs, int64_t rec_cap,
                         int64_t *nrec);
/* The same, asynchronous: one caller keeps many chunks in flight, as the reference's reader keeps 32
 * partitions queued (LazyFileReader.cs:14) for its tasks.  submit queues the request and returns a
 * ticket at once; a launcher thread of the ctx (started by the first submit) combines the queued
 * requests -- a burst of submissions goes into one launch of up to 256 chunks --, a copier thread
 * copies each decoded chunk's bytes / records into the buffers given at submit (up to 8 threads per
 * launch) while the next launch runs, and ppg_decompress_chunk_wait blocks until that is done,
 * returns the status and counts, and frees the ticket (slice, out and recs must stay valid until
 * then).  Every ticket must be waited for, each once, on the ctx it was submitted to.  (Both forms:
 * where results of a launch are copied out together, the whole 2 MiB pages inside each caller
 * buffer get madvise(MADV_HUGEPAGE) first -- advice only, the copy is ~2x faster into fresh pages.) */
typedef struct ppg_chunk_req ppg_chunk_req;
int ppg_decompress_chunk_submit(ppg_ctx *ctx, const ppg_index *ix, int32_t k, const uint8_t *slice, int64_t slice_len,
                                uint8_t *out, int64_t out_cap, uint32_t *recs, int64_t rec_cap, ppg_chunk_req **req);
int ppg_decompress_chunk_wait(ppg_ctx *ctx, ppg_chunk_req *req, int64_t *produced, int64_t *nrec);
/* ppg_decompress_chunk (and _submit) calls on this ctx so far, the launches that served them, the
 * most calls one launch served. */
int ppg_decompress_chunk_stats(ppg_ctx *ctx, int64_t *calls, int64_t *launches, int64_t *max_batch);
/* Chunks split by the search for inner block starts above, and the side points it found. */
int ppg_decompress_chunk_split_stats(ppg_ctx *ctx, int64_t *chunks, int64_t *side_points);

/* ======================= DecompressAll over a shard (README "DecompressAll") =======================
 * A shard is chunks [first, first+n) of an index, with their compressed bytes resident on the
 * ctx's GPU: comp holds file bytes [Index[first].Input-1, Index[first+n].Input-1]
 * (comp_len = Index[first+n].Input - Index[first].Input + 1).  comp_on_device != 0 means comp
 * is already a device pointer on this GPU (4-byte aligned, readable 64 bytes past comp_len);
 * otherwise it is copied.  out_capacity bounds the device output buffer: chunks are decoded
 * in batches whose outputs fit, the buffer being reused (0 = whole shard at once). */
typedef struct ppg_shard ppg_shard;

int ppg_shard_create(ppg_ctx *ctx, const ppg_index *ix, int32_t first, int32_t n, const void *comp, int64_t comp_len,
                     int comp_on_device, int64_t out_capacity, ppg_shard **out);
void ppg_shard_free(ppg_shard *sh);

/* Inflate + parse every chunk of the shard (BatchedFASTQ's populateCache body, BatchedFASTQ.cs:
 * 63-74, for all chunks).  Returns 0, or the first chunk error (ZResult code).  Blocking. */
int ppg_shard_run(ppg_shard *sh);

/* Parallelism inside chunks (no reference counterpart: the reference decodes a chunk on one
 * thread, Core.cs:133-192; SURVEY §8f #1 "a denser side-index for sub-chunk parallelism").
 * nsub side points, sorted by output, each a deflate block start strictly inside one of the
 * shard's chunks: absolute file bit position (8*Input - Bits in Point terms), absolute output
 * offset, and the 32 KiB of output before it (host array, nsub * 32768 bytes).  Later runs decode
 * each chunk as one wave per piece between its Point, its side points and the next Point, and
 * fold the pieces back into the chunk (ppg_split_merge): results, records and bytes are
 * identical to the unsplit run.  A side point that is not where the previous piece's blocks end
 * fails the chunk with PPG_DATA_ERROR.  Works with any number of output batches (each batch
 * launches its chunks' pieces); nsub = 0 restores one wave per chunk. */
int ppg_shard_set_split(ppg_shard *sh, int32_t nsub, const int64_t *bit, const int64_t *output,
                        const uint8_t *windows);

/* Per-chunk results of the last run (host arrays of length n; any may be NULL). */
int ppg_shard_results(ppg_shard *sh, int64_t *records, int64_t *produced, int32_t *status, int32_t *flags,
                      int64_t *end_bit);
int64_t ppg_shard_total_records(ppg_shard *sh);
int32_t ppg_shard_batches(ppg_shard *sh);

/* Chunk bytes (only when the shard ran as one batch: the output buffer is reused by the next
 * batch; ppg_cursor streams bytes of any size) / record descriptors (any number of batches: the
 * descriptors of every batch stay resident) to the host.
 * Descriptor j of chunk k = 4 uint32 (n1,n2,n3,n4) relative to raw_k = offset_k ++ chunk_k:
 * Identifier=[r+1,n1) Sequence=[n1+1,n2) Other=[n2+2,n3) Quality=[n3+1,n4), where r = 0 for
 * the chunk's first record and the previous n4+1 otherwise (Parsing.cs:11-51). */
int ppg_shard_copy_chunk(ppg_shard *sh, int32_t k, uint8_t *dst, int64_t cap, int64_t *len);
int ppg_shard_copy_records(ppg_shard *sh, int32_t k, uint32_t *dst, int64_t cap, int64_t *nrec);
int ppg_shard_record_base(ppg_shard *sh, int64_t *base); /* n record bases (exclusive scan) */
/* Bytes [off, off+len) of a one-batch shard's decompressed output (off relative to
 * Index[first].Output; chunks are contiguous) into host memory or (dst_on_device) device memory
 * on this GPU, on the ctx stream. */
int ppg_shard_copy_output(ppg_shard *sh, int64_t off, int64_t len, void *dst, int dst_on_device);

/* Paired reads (the reference only names the goal, README.md:9): the spot number
 * of every record of a one-batch shard, in record order, into caller device memory (cap int64s):
 * the digits between the first two '.' of the Identifier ("SRR<id>.<spot>.<mate> ..."), -1 when
 * absent, -2 for a record the reference parses twice, which a pairing drops. */
int ppg_shard_keys(ppg_shard *sh, int64_t *dev_keys, int64_t cap);
/* The same keys for a shard of any number of batches: from the next ppg_shard_run on, each batch
 * writes its records' keys to dev_keys[shard record number] (caller device memory on this GPU, cap
 * entries) on the ctx stream while its output is resident.  NULL / 0 turns it off.  A run with
 * more records than cap fails with PPG_BUF_ERROR. */
int ppg_shard_set_keys(ppg_shard *sh, int64_t *dev_keys, int64_t cap);

/* Whether the last ppg_shard_run of the shard filled the ppg_shard_set_keys buffer (1) or not (0:
 * none attached, attached after that run, or the run failed). */
int ppg_shard_keys_ready(ppg_shard *sh);

/* Device-resident per-chunk record counts (int64[n]) copied to caller device memory on this
 * GPU (the input of the cross-GPU all-gather). */
int ppg_shard_counts_to_device(ppg_shard *sh, int64_t *dev_dst);

/* Device time of the last run, from hipEvents on the ctx stream: inflate kernels only, parse
 * kernels only, and the whole run (ms). */
int ppg_shard_timing(ppg_shard *sh, float *inflate_ms, float *parse_ms, float *total_ms);

/* =============== DecompressAll from a .gz file: host ingest (LazyFileReader.cs:10-98) ===============
 * Streams chunks [first, first+n) of gz_path through the GPU: `threads` reader threads (0 = 8)
 * pread pieces of about piece_bytes compressed bytes (0 = 8 GiB: a launch needs thousands of
 * chunks to fill the GPU) into pinned host buffers; a copy stream moves each piece to HBM and a
 * helper thread prepares its jobs/windows while the previous piece decodes, so page cache, PCIe
 * and the kernels overlap.  Buffers persist in the ctx across calls.  records[i] (may be NULL) receives chunk first+i's record count,
 * *total_records their sum, *seconds the wall time from the first read to the last result.
 * Returns 0, PPG_IO_ERROR for an unreadable file, or the first chunk error (ZResult code). */
int ppg_file_decompress_all(ppg_ctx *ctx, const ppg_index *ix, const char *gz_path, int32_t first, int32_t n,
                            int64_t piece_bytes, int threads, int64_t *records, int64_t *total_records,
                            double *seconds);
/* Frees the buffers ppg_file_decompress_all keeps in the ctx (its device pieces and their shards'
 * outputs, tens of GB at 8 GiB pieces; the pinned staging; its streams) -- e.g. before other work
 * needs the HBM; the next call allocates them again.  Not while a ppg_file_decompress_all runs on
 * the ctx.  Returns 0, or PPG_ARG_ERROR for a NULL ctx. */
int ppg_file_release(ppg_ctx *ctx);

/* ======================= streamed records: BatchedFASTQ's enumerator =======================
 * Decompressor/BatchedFASTQ.cs:29-101 (IEnumerable<FastqRecord> over a bounded record cache fed by
 * LazyFileReader's partition queue, LazyFileReader.cs:41-97) over the GPU path, in bounded memory:
 * chunks [first, first+n) of gz_path in batches of whole chunks of at most batch_bytes of text
 * (0 = 1 GiB; a single larger chunk is its own batch).  Up to five batches are in flight, each in a
 * slot sized once at open for the largest batch: per slot ~1.13 x batch text + its compressed bytes
 * of pinned host memory and ~1.4-2.4 x that text of HBM (8 GiB batches: ~55 GB pinned in all); the
 * slot count drops (to 2 at least) where that would exceed half the available host memory or 80%
 * of the free HBM.  Each batch is pread (`threads` readers)
 * into pinned memory, decoded on the GPU and handed back as host memory: the chunks' raw bytes
 * raw_k = offset_k ++ chunk_k (Parsing.cs's CombinedMemory) concatenated in `text` at raw_off[k],
 * and the records of chunk k as desc[4*j .. 4*j+3] for j in [rec_off[k], rec_off[k+1]), each the
 * newline positions (n1,n2,n3,n4) relative to raw_k with the field slices of ppg_shard_copy_records.
 * While the caller walks batch k the library reads and decodes batch k+1; a batch is valid until
 * the next ppg_cursor_next (a FastqRecord is invalid after the next MoveNext, BatchedFASTQ.cs:56).
 * Order is canonical (chunk by chunk), not the reference's interleaving. */
typedef struct ppg_cursor ppg_cursor;
typedef struct {
    int32_t first_chunk;      /* index chunk of the batch's first chunk */
    int32_t nchunks;
    int64_t record_base;      /* records handed out by this cursor before this batch */
    int64_t nrecords;
    const uint8_t *text;      /* raw_k at text + raw_off[k] */
    const int64_t *raw_off;   /* nchunks + 1 entries */
    const uint32_t *desc;     /* 4 per record */
    const int64_t *rec_off;   /* nchunks + 1 entries */
} ppg_batch;

int ppg_cursor_open(ppg_ctx *ctx, const ppg_index *ix, const char *gz_path, int32_t first, int32_t n,
                    int64_t batch_bytes, int threads, ppg_cursor **out);
/* PPG_OK with the next batch in *b, PPG_STREAM_END after the last one, or a ZResult error. */
int ppg_cursor_next(ppg_cursor *c, ppg_batch *b);
int32_t ppg_cursor_batches(const ppg_cursor *c);
void ppg_cursor_close(ppg_cursor *c);

/* ======================= multi-GPU DecompressAll (one process per GPU) =======================
 * BatchedFASTQ's fan-out (BatchedFASTQ.cs:62-77: a task per chunk) becomes a fan-out over GPUs:
 * rank r decodes the contiguous chunk range [bounds[r], bounds[r+1]) that ppg_partition balances
 * by compressed bytes, with no exchange on the data path; the one collective is an all-gather of
 * per-chunk record counts (padded to the widest range: RCCL has no all-gatherv) followed by an
 * exclusive scan, giving every chunk its global record number.
 *
 * A ppg_comm is an RCCL communicator (ncclAllGather on the ctx stream, over xGMI) -- made by the
 * library from a unique id that rank 0 creates and the host hands to every rank (ppg_comm_init),
 * or wrapping the caller's ncclComm_t (ppg_comm_from_rccl) -- or a host shared-memory transport
 * between processes of one machine (ppg_comm_init_host; name = "/something", unique per job):
 * RCCL refuses two ranks on one GPU, so that is how the N > 1 path is rehearsed on one GPU.
 * librccl is loaded at run time (dlopen librccl.so.1: the copy already in the process, if any).
 * A rank that fails still joins the gather, and every rank then returns the first failing
 * rank's status, so an error never leaves the others waiting. */
typedef struct ppg_comm ppg_comm;
#define PPG_COMM_ID_BYTES 128
int ppg_comm_unique_id(uint8_t *id);   /* PPG_COMM_ID_BYTES bytes (ncclGetUniqueId) */
int ppg_comm_init(ppg_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t *id, ppg_comm **out);
int ppg_comm_from_rccl(ppg_ctx *ctx, void *nccl_comm, int32_t nranks, int32_t rank, ppg_comm **out);
int ppg_comm_init_host(int32_t nranks, int32_t rank, const char *name, ppg_comm **out);
int ppg_comm_rank(const ppg_comm *c, int32_t *rank, int32_t *nranks);
void ppg_comm_free(ppg_comm *c);
int ppg_rccl_version(int *version);    /* ncclGetVersion of the librccl in use */

/* All-to-all-v of int64 values: counts[src * nranks + dst] values go from rank src to rank dst
 * (the whole matrix, the same on every rank); send holds this rank's outgoing values by
 * destination, recv receives by source, both in rank order.  RCCL: device buffers on the comm's GPU
 * (on_device = 1; grouped ncclSend / ncclRecv over xGMI); host transport: host or device buffers,
 * moved through shared memory in rounds.  The exchange step of ppg_pairs_check. */
int ppg_comm_alltoallv(ppg_comm *c, const int64_t *send, int64_t *recv, const int64_t *counts, int on_device);

/* bounds[0..nranks]: rank r owns chunks [bounds[r], bounds[r+1]) of [first, first+n) */
int ppg_partition(const ppg_index *ix, int32_t first, int32_t n, int32_t nranks, int32_t *bounds);
/* After ppg_shard_run of this rank's shard (chunks [bounds[rank], bounds[rank+1])): the count
 * all-gather + scan.  counts / bases (may be NULL): bounds[nranks] - bounds[0] entries. */
int ppg_shard_gather_counts(ppg_shard *sh, ppg_comm *comm, const int32_t *bounds, int64_t *counts, int64_t *bases,
                            int64_t *total_records);
/* The whole path for a C# host's BatchedFASTQ.Count() over N GPUs: partition the index's chunks,
 * pread this rank's compressed range from gz_path, decode it (out_capacity as ppg_shard_create),
 * gather.  counts / bases (may be NULL): Count-1 entries in canonical order. */
int ppg_dist_decompress_all(ppg_ctx *ctx, ppg_comm *comm, const ppg_index *ix, const char *gz_path,
                            int64_t out_capacity, int64_t *counts, int64_t *bases, int64_t *total_records);

/* ============ paired reads: R1 / R2 shards checked record by record ============
 * The reference only names the goal (README.md:9).  Pair number i = the i-th record of R1 and of
 * R2 after dropping the records the reference parses twice (key -2); a pair is good when
 * both spot keys (ppg_shard_keys) are present and equal.  ppg_pairs_check runs on the device: the
 * shards' keys (their ppg_shard_set_keys buffers when the last run filled them, else extracted now
 * from one-batch shards), the duplicates dropped through a map, the keys compared.  With a comm
 * (N ranks; rank r holds R1 and R2 shards of its own contiguous chunk ranges, which do not line up
 * between the files) pairs are owned evenly by pair number and every key moves to its owner: a
 * status + count all-gather, one all-to-all-v per file (RCCL ncclSend / ncclRecv, or the host
 * transport), the compare, a result all-gather; every rank gets the same result and a failing rank
 * never leaves the others waiting.  Both shards (and an RCCL comm) must be on one GPU.  A ppg_pairs
 * keeps its device scratch across checks. */
typedef struct {
    int64_t pairs;            /* min of the two files' records after dropping duplicates */
    int64_t records[2];       /* R1 / R2 records after dropping duplicates (all ranks) */
    int64_t duplicates[2];    /* Q1 duplicates dropped (this rank) */
    int64_t mismatches;       /* pairs whose keys differ or are missing (< 0), + |records[0] - records[1]| */
    int64_t first_bad;        /* the first such pair number, or -1 */
    int64_t first_keys[2];    /* its R1 / R2 spot keys (-1 when a file has no such record) */
} ppg_pair_result;
typedef struct ppg_pairs ppg_pairs;
int ppg_pairs_create(ppg_pairs **out);
int ppg_pairs_check(ppg_pairs *p, ppg_shard *r1, ppg_shard *r2, ppg_comm *comm, ppg_pair_result *result);
/* After a check: the shard record numbers (this rank's shard of `file`, 0 = R1) of pair numbers
 * [lo, hi), -1 for pairs whose record another rank holds -- record-aligned pair chunks are pair
 * numbers [j*K, (j+1)*K); the records themselves via ppg_shard_record_base / ppg_shard_copy_records. */
int ppg_pairs_records(const ppg_pairs *p, int32_t file, int64_t lo, int64_t hi, int64_t *shard_record);
void ppg_pairs_free(ppg_pairs *p);

/* ---- record-aligned pair chunks (BASELINE configs[4]: "chunk=50 000, record-aligned
 * pair chunks"; the reference's goal, README.md:9) ----
 * After ppg_pairs_check: pair chunk j = pairs [j*K, min((j+1)*K, pairs)).  Each half (file 0 = R1,
 * 1 = R2) is packed contiguously on the device: its records' bytes back to back -- each record from
 * its '@' to its quality line's '\n', the FastqRecord copy of Parsing.cs:41-47 -- and one 16-B
 * descriptor (n1, n2, n3, n4: the record's newline positions) per record, relative to the half's
 * first byte: the layout of one chunk's raw text + descriptors, so the same record reader applies
 * (record i starts at n4[i-1] + 1, record 0 at 0).
 *  ppg_pairs_emit_begin  the plan for this rank's pair chunks, on the shards and comm of the check.
 *      One rank: every pair chunk, in windows of at most window_bytes per half-file (0: 8 GiB; one
 *      pair chunk at least).  Multi-batch shards (configs[4]'s 2 x 25 GB on one GPU) have their
 *      batches run again as the windows advance -- both files' together, each on its own stream --
 *      and a pair chunk that straddles a batch boundary is carried across; nothing else may run the
 *      shards until the emission is done.  N ranks: rank r owns the pair chunks that start in its
 *      R1 range; the shards must be one-batch (resident; else PPG_UNSUPPORTED).
 *  ppg_pairs_emit_run    one rank, no check first: the emission drives the shards' own run.  Both
 *      shards carry a keys buffer (ppg_shard_set_keys); their batches run once each, in order, as
 *      the windows advance -- each batch's records numbered (its Q1 duplicates found from its keys)
 *      and packed while it is resident, so a multi-batch shard is decoded once, not twice.  After
 *      the last window (PPG_STREAM_END) both shards stand as ppg_shard_run leaves them and
 *      ppg_pairs_check follows (it may report mismatches the windows already emitted).  A caller
 *      that stops early leaves the shards unrun.
 *  ppg_pairs_emit_next   packs the next window of this rank's pair chunks [*j0, *j1) on the device;
 *      PPG_STREAM_END when there is none.  N ranks: the first call is collective (every rank calls
 *      it: the records a rank does not hold move from their ranks over ppg_comm_alltoallv -- RCCL
 *      ncclSend / ncclRecv over xGMI, or the host transport) and is the rank's one window.
 *      A half's descriptors are 32-bit positions, so a half of 4 GiB or more (pair_chunk of ~11 M
 *      150 bp records) is PPG_UNSUPPORTED, before anything of it is packed (N ranks: agreed in the
 *      exchange's status gather, or after the exchange).  PPG_DATA_ERROR if the shards' batches cannot
 *      complete a pair chunk (never expected: the emission ends instead of looping).
 *  ppg_pairs_chunk       device pointers of a half of the current window (valid until the next call).
 *  ppg_pairs_copy_chunk  a half into caller memory (bytes and/or descriptors; NULL skips).
 *  ppg_pairs_emit_stats  [0] ms (re-)running batches, [1] ms packing, [2] ms exchanging, [3] ms in
 *      emit_next, [4] batches re-run, [5] pair chunks in all, [6..7] this rank's [j_lo, j_hi)
 *      (N ranks: after the exchange; emit_run: [5] and [7] once the last window is out). */
int ppg_pairs_emit_begin(ppg_pairs *p, ppg_shard *r1, ppg_shard *r2, ppg_comm *comm, int64_t pair_chunk,
                         int64_t window_bytes);
int ppg_pairs_emit_run(ppg_pairs *p, ppg_shard *r1, ppg_shard *r2, int64_t pair_chunk, int64_t window_bytes);
int ppg_pairs_emit_next(ppg_pairs *p, int64_t *j0, int64_t *j1);
int ppg_pairs_chunk(ppg_pairs *p, int64_t j, int32_t file, const uint8_t **bytes, int64_t *len, const uint32_t **desc,
                    int64_t *nrec);
int ppg_pairs_copy_chunk(ppg_pairs *p, int64_t j, int32_t file, uint8_t *dst, int64_t cap, int64_t *len, uint32_t *desc,
                         int64_t desc_cap, int64_t *nrec);
int ppg_pairs_emit_stats(const ppg_pairs *p, double *vals, int32_t n);

/* Library build string (kernel ISA, version). */
const char *ppg_version(void);
/* "inflate-<16 hex>": a hash of the inflate kernels' object (all variants + launcher), fixed at
 * build time.  Measurements quoted from files (bench.py's roofline.traffic) carry it and are
 * refused when it differs from the library in use. */
const char *ppg_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* PPGPU_H */

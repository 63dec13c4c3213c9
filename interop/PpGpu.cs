// interop/PpGpu.cs — the P/Invoke class a maintainer adds next to the reference's LibZ
// (Interop/PlatformInterop.cs:6-35) to bind libppgpu.so.  One extern per entry point of
// include/ppgpu.h, same argument order and meaning; status codes keep ZResult's values
// (Interop/Conventions.cs:9-20) plus the library codes in PpgStatus.  (Source only: this image
// has no .NET SDK, so it is not compiled here; tests/test_interop_cs.py checks it covers the
// header exactly.)
using System.Runtime.InteropServices;

namespace ParallelParsing.Interop;

public static class PpgStatus
{
    public const int IndexOutOfRange = -50;   // C# IndexOutOfRangeException (SURVEY Q4, Core.cs:93)
    public const int IoError = -51;
    public const int ArgError = -52;
    public const int Unsupported = -53;
    public const int DeviceError = -100;
    public const int NoDevice = -101;
}

/// <summary>A libppgpu failure that is not a zlib result (PpgStatus codes other than
/// IndexOutOfRange): bad arguments, unreadable files, unsupported input, device errors.  zlib's
/// results keep the reference's ZException (Interop/Conventions.cs:33-41).</summary>
public class PpgException : Exception
{
    public int Code { get; }

    public PpgException(int code, string what) : base($"libppgpu: {what} ({code})")
    {
        Code = code;
    }
}

[StructLayout(LayoutKind.Sequential)]
public unsafe struct PpgBatch          // ppg_batch
{
    public int FirstChunk;
    public int NChunks;
    public long RecordBase;
    public long NRecords;
    public byte* Text;                  // raw_k = offset_k ++ chunk_k at Text + RawOff[k]
    public long* RawOff;                // NChunks + 1
    public uint* Desc;                  // (n1, n2, n3, n4) per record, relative to raw_k
    public long* RecOff;                // NChunks + 1
}

[StructLayout(LayoutKind.Sequential)]
public unsafe struct PpgPairResult     // ppg_pair_result
{
    public long Pairs;
    public fixed long Records[2];
    public fixed long Duplicates[2];
    public long Mismatches;
    public long FirstBad;
    public fixed long FirstKeys[2];
}

internal static unsafe class PpGpu
{
    const string Lib = "ppgpu";   // libppgpu.so from parallelparsing_amd/

    // ---- Index: Common/Index.cs, Common/IndexIO.cs, Core.BuildDeflateIndex (Core.cs:14-131) ----
    [DllImport(Lib)] public static extern int ppg_index_build_file(string gzPath, uint chunksize, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_build_mem(byte* gz, long gzLen, uint chunksize, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_build_gpu(nint ctx, byte* gz, long gzLen, int gzOnDevice,
        uint chunksize, long pieceBytes, long outCapacity, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_build_gpu_side(nint ctx, byte* gz, long gzLen, int gzOnDevice,
        uint chunksize, long pieceBytes, long outCapacity, long sideBytes, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_side_count(nint ix);
    [DllImport(Lib)] public static extern int ppg_index_side_points(nint ix, long* bit, long* output, byte* windows);
    [DllImport(Lib)] public static extern int ppg_index_set_side_points(nint ix, int n, long* bit, long* output,
        byte* windows);
    [DllImport(Lib)] public static extern int ppg_index_build_gpu_file(nint ctx, string gzPath, uint chunksize,
        long pieceBytes, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_build_gpu_stats(nint ctx, double* vals, int n);
    [DllImport(Lib)] public static extern int ppg_index_serialize(nint ix, string path);
    [DllImport(Lib)] public static extern int ppg_index_deserialize(string path, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_from_points(int count, long* output, long* input, int* bits,
        byte* windows, int* offsetLen, byte* offsets, int chunkMaxBytes, out nint ix);
    [DllImport(Lib)] public static extern int ppg_index_count(nint ix);
    [DllImport(Lib)] public static extern int ppg_index_chunk_max_bytes(nint ix);
    [DllImport(Lib)] public static extern int ppg_index_point(nint ix, int i, out long output, out long input,
        out int bits, out int offsetLen);
    [DllImport(Lib)] public static extern byte* ppg_index_window(nint ix, int i);
    [DllImport(Lib)] public static extern byte* ppg_index_offset(nint ix, int i);
    [DllImport(Lib)] public static extern void ppg_index_free(nint ix);
    [DllImport(Lib)] public static extern int ppg_index_validate(nint ix, int first, int n);

    // ---- device context: one per GPU ----
    [DllImport(Lib)] public static extern int ppg_device_count(out int n);
    [DllImport(Lib)] public static extern int ppg_open(int device, out nint ctx);
    [DllImport(Lib)] public static extern void ppg_close(nint ctx);
    [DllImport(Lib)] public static extern nint ppg_ctx_stream(nint ctx);
    [DllImport(Lib)] public static extern int ppg_ctx_wait_stream(nint ctx, nint stream);
    [DllImport(Lib)] public static extern int ppg_stream_wait_ctx(nint ctx, nint stream);

    // ---- README "Decompress": Core.ExtractDeflateIndex (Core.cs:133-192) + Parsing.Parse ----
    [DllImport(Lib)] public static extern int ppg_decompress_chunk(nint ctx, nint ix, int k, byte* slice,
        long sliceLen, byte* output, long outCap, out long produced, uint* recs, long recCap, out long nrec);
    // asynchronous Decompress: many chunks in flight from one caller (ppg_decompress_chunk_submit / _wait)
    [DllImport(Lib)] public static extern int ppg_decompress_chunk_submit(nint ctx, nint ix, int k, byte* slice,
        long sliceLen, byte* outp, long outCap, uint* recs, long recCap, out nint req);
    [DllImport(Lib)] public static extern int ppg_decompress_chunk_wait(nint ctx, nint req, out long produced,
        out long nrec);
    [DllImport(Lib)] public static extern int ppg_decompress_chunk_stats(nint ctx, out long calls, out long launches,
        out long maxBatch);
    [DllImport(Lib)] public static extern int ppg_decompress_chunk_split_stats(nint ctx, out long chunks,
        out long sidePoints);

    // ---- README "DecompressAll": a shard of chunks resident on one GPU ----
    [DllImport(Lib)] public static extern int ppg_shard_create(nint ctx, nint ix, int first, int n, byte* comp,
        long compLen, int compOnDevice, long outCapacity, out nint shard);
    [DllImport(Lib)] public static extern void ppg_shard_free(nint shard);
    [DllImport(Lib)] public static extern int ppg_shard_run(nint shard);
    [DllImport(Lib)] public static extern int ppg_shard_set_split(nint shard, int nsub, long* bit, long* output,
        byte* windows);
    [DllImport(Lib)] public static extern int ppg_shard_results(nint shard, long* records, long* produced,
        int* status, int* flags, long* endBit);
    [DllImport(Lib)] public static extern long ppg_shard_total_records(nint shard);
    [DllImport(Lib)] public static extern int ppg_shard_batches(nint shard);
    [DllImport(Lib)] public static extern int ppg_shard_copy_chunk(nint shard, int k, byte* dst, long cap, out long len);
    [DllImport(Lib)] public static extern int ppg_shard_copy_records(nint shard, int k, uint* dst, long cap,
        out long nrec);
    [DllImport(Lib)] public static extern int ppg_shard_record_base(nint shard, long* b);
    [DllImport(Lib)] public static extern int ppg_shard_copy_output(nint shard, long off, long len, void* dst,
        int dstOnDevice);
    [DllImport(Lib)] public static extern int ppg_shard_keys(nint shard, long* devKeys, long cap);
    [DllImport(Lib)] public static extern int ppg_shard_set_keys(nint shard, long* devKeys, long cap);
    [DllImport(Lib)] public static extern int ppg_shard_keys_ready(nint shard);
    [DllImport(Lib)] public static extern int ppg_shard_counts_to_device(nint shard, long* devDst);
    [DllImport(Lib)] public static extern int ppg_shard_timing(nint shard, out float inflateMs, out float parseMs,
        out float totalMs);

    // ---- LazyFileReader (LazyFileReader.cs:10-98): DecompressAll straight from the file ----
    [DllImport(Lib)] public static extern int ppg_file_decompress_all(nint ctx, nint ix, string gzPath, int first,
        int n, long pieceBytes, int threads, long* records, out long totalRecords, out double seconds);
    [DllImport(Lib)] public static extern int ppg_file_release(nint ctx);

    // ---- BatchedFASTQ's enumerator (BatchedFASTQ.cs:29-101): streamed record batches ----
    [DllImport(Lib)] public static extern int ppg_cursor_open(nint ctx, nint ix, string gzPath, int first, int n,
        long batchBytes, int threads, out nint cursor);
    [DllImport(Lib)] public static extern int ppg_cursor_next(nint cursor, out PpgBatch batch);
    [DllImport(Lib)] public static extern int ppg_cursor_batches(nint cursor);
    [DllImport(Lib)] public static extern void ppg_cursor_close(nint cursor);

    // ---- multi-GPU DecompressAll: partition + count all-gather over RCCL inside the library ----
    [DllImport(Lib)] public static extern int ppg_comm_unique_id(byte* id /* 128 bytes */);
    [DllImport(Lib)] public static extern int ppg_comm_init(nint ctx, int nranks, int rank, byte* id, out nint comm);
    [DllImport(Lib)] public static extern int ppg_comm_from_rccl(nint ctx, nint ncclComm, int nranks, int rank,
        out nint comm);
    [DllImport(Lib)] public static extern int ppg_comm_init_host(int nranks, int rank, string name, out nint comm);
    [DllImport(Lib)] public static extern int ppg_comm_rank(nint comm, out int rank, out int nranks);
    [DllImport(Lib)] public static extern void ppg_comm_free(nint comm);
    [DllImport(Lib)] public static extern int ppg_rccl_version(out int version);
    [DllImport(Lib)] public static extern int ppg_comm_alltoallv(nint comm, long* send, long* recv, long* counts,
        int onDevice);
    [DllImport(Lib)] public static extern int ppg_partition(nint ix, int first, int n, int nranks, int* bounds);
    [DllImport(Lib)] public static extern int ppg_shard_gather_counts(nint shard, nint comm, int* bounds,
        long* counts, long* bases, out long totalRecords);
    [DllImport(Lib)] public static extern int ppg_dist_decompress_all(nint ctx, nint comm, nint ix, string gzPath,
        long outCapacity, long* counts, long* bases, out long totalRecords);

    // ---- paired reads (SURVEY §8f #3, README.md:9): R1 / R2 shards checked on the device ----
    [DllImport(Lib)] public static extern int ppg_pairs_create(out nint pairs);
    [DllImport(Lib)] public static extern int ppg_pairs_check(nint pairs, nint r1, nint r2, nint comm,
        out PpgPairResult result);
    [DllImport(Lib)] public static extern int ppg_pairs_records(nint pairs, int file, long lo, long hi,
        long* shardRecord);
    [DllImport(Lib)] public static extern void ppg_pairs_free(nint pairs);
    // record-aligned pair chunks, packed on the device (ppg_pairs_emit_*)
    [DllImport(Lib)] public static extern int ppg_pairs_emit_begin(nint pairs, nint r1, nint r2, nint comm,
        long pairChunk, long windowBytes);
    [DllImport(Lib)] public static extern int ppg_pairs_emit_run(nint pairs, nint r1, nint r2, long pairChunk,
        long windowBytes);
    [DllImport(Lib)] public static extern int ppg_pairs_emit_next(nint pairs, out long j0, out long j1);
    [DllImport(Lib)] public static extern int ppg_pairs_chunk(nint pairs, long j, int file, out nint bytes, out long len,
        out nint desc, out long nrec);
    [DllImport(Lib)] public static extern int ppg_pairs_copy_chunk(nint pairs, long j, int file, byte* dst, long cap,
        out long len, uint* desc, long descCap, out long nrec);
    [DllImport(Lib)] public static extern int ppg_pairs_emit_stats(nint pairs, double* vals, int n);

    [DllImport(Lib)] public static extern nint ppg_version();
    [DllImport(Lib)] public static extern nint ppg_build_id();

    // Status -> exception, as the reference's callers do (Core.cs:31-34, :68-74, :178-179): zlib's
    // ZResult codes (Conventions.cs:9-20) become ZException; the IndexOutOfRange that CreateIndex's
    // offset buffer throws in the reference (Core.cs:93, SURVEY Q4) stays IndexOutOfRangeException;
    // every library code becomes a PpgException carrying it.  Every PPG_* status of ppgpu.h has a
    // case here (tests/test_interop_cs.py); an unknown code is a PpgException too, never a ZResult
    // cast of a value the enum does not define.
    public static void Check(int rc)
    {
        switch (rc)
        {
            case 0: return;                                                       // PPG_OK
            case 1: throw new ZException(ZResult.STREAM_END);                     // PPG_STREAM_END
            case 2: throw new ZException(ZResult.NEED_DICT);                      // PPG_NEED_DICT
            case -1: throw new ZException(ZResult.ERRNO);                         // PPG_ERRNO
            case -2: throw new ZException(ZResult.STREAM_ERROR);                  // PPG_STREAM_ERROR
            case -3: throw new ZException(ZResult.DATA_ERROR);                    // PPG_DATA_ERROR
            case -4: throw new ZException(ZResult.MEM_ERROR);                     // PPG_MEM_ERROR
            case -5: throw new ZException(ZResult.BUF_ERROR);                     // PPG_BUF_ERROR
            case -6: throw new ZException(ZResult.VERSION_ERROR);                 // PPG_VERSION_ERROR
            case -50: throw new IndexOutOfRangeException();                       // PPG_INDEX_OUT_OF_RANGE
            case -51: throw new PpgException(rc, "I/O error");                    // PPG_IO_ERROR
            case -52: throw new PpgException(rc, "invalid argument");             // PPG_ARG_ERROR
            case -53: throw new PpgException(rc, "unsupported input");            // PPG_UNSUPPORTED
            case -100: throw new PpgException(rc, "device error");                // PPG_DEVICE_ERROR
            case -101: throw new PpgException(rc, "no gfx950 device");            // PPG_NO_DEVICE
            default: throw new PpgException(rc, "unknown status");
        }
    }
}

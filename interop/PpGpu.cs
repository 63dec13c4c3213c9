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
    public const int IndexOutOfRange = -50;   // C# IndexOutOfRangeException (SURVEY Q4)
    public const int IoError = -51;
    public const int ArgError = -52;
    public const int Unsupported = -53;
    public const int DeviceError = -100;
    public const int NoDevice = -101;
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
    [DllImport(Lib)] public static extern int ppg_shard_counts_to_device(nint shard, long* devDst);
    [DllImport(Lib)] public static extern int ppg_shard_timing(nint shard, out float inflateMs, out float parseMs,
        out float totalMs);

    // ---- LazyFileReader (LazyFileReader.cs:10-98): DecompressAll straight from the file ----
    [DllImport(Lib)] public static extern int ppg_file_decompress_all(nint ctx, nint ix, string gzPath, int first,
        int n, long pieceBytes, int threads, long* records, out long totalRecords, out double seconds);

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
    [DllImport(Lib)] public static extern int ppg_partition(nint ix, int first, int n, int nranks, int* bounds);
    [DllImport(Lib)] public static extern int ppg_shard_gather_counts(nint shard, nint comm, int* bounds,
        long* counts, long* bases, out long totalRecords);
    [DllImport(Lib)] public static extern int ppg_dist_decompress_all(nint ctx, nint comm, nint ix, string gzPath,
        long outCapacity, long* counts, long* bases, out long totalRecords);

    [DllImport(Lib)] public static extern nint ppg_version();
    [DllImport(Lib)] public static extern nint ppg_build_id();

    public static void Check(int rc)
    {
        if (rc != 0) throw new ZException((ZResult)rc);   // as Core.cs:68-74 / :178-179
    }
}

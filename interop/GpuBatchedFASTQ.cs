// interop/GpuBatchedFASTQ.cs — Decompressor/BatchedFASTQ.cs:10-101's IEnumerable<FastqRecord>
// surface over libppgpu (interop/PpGpu.cs).  Same constructors, same Count() / enumeration use
// as Decompressor/Program.cs:48-52; the records are those Parsing.Parse cuts (Parsing.cs:11-51),
// in canonical chunk order (the reference interleaves producers, SURVEY Q5).
//
//  * enumeration: ppg_cursor streams the file in batches of whole chunks (bounded memory, like
//    RECORD_CACHE_MAX_LENGTH + LazyFileReader's partition queue); each batch's raw bytes are copied
//    into one managed array that the batch's FastqRecords slice (a record stays valid after the
//    next MoveNext here; the reference invalidates it, Q9);
//  * Count(): ppg_file_decompress_all on one GPU, or ppg_dist_decompress_all when the process is
//    one rank of a multi-GPU job (GpuJob: the ranks' RCCL communicator);
//  * a rank of a multi-GPU job enumerates its own share (ppg_partition's chunk range).
// (Source only: no .NET SDK in this image; tests/test_interop_cs.py checks the externs it uses.)
using System;
using System.Collections;
using ParallelParsing.Common;
using ParallelParsing.Interop;
using Index = ParallelParsing.Common.Index;

namespace ParallelParsing;

/// <summary>One rank of a multi-GPU DecompressAll: a device context and an RCCL communicator.</summary>
public sealed unsafe class GpuJob : IDisposable
{
    public nint Ctx { get; }
    public nint Comm { get; }
    public int Rank { get; }
    public int NRanks { get; }

    /// <param name="uniqueId">128 bytes from <see cref="NewUniqueId"/> on rank 0, sent to every rank
    /// by the host's own launcher (MPI, a file, a socket).</param>
    public GpuJob(int device, int nranks, int rank, byte[] uniqueId)
    {
        PpGpu.Check(PpGpu.ppg_open(device, out var ctx));
        Ctx = ctx;
        nint comm;
        fixed (byte* id = uniqueId) PpGpu.Check(PpGpu.ppg_comm_init(ctx, nranks, rank, id, out comm));
        Comm = comm;
        Rank = rank;
        NRanks = nranks;
    }

    public static byte[] NewUniqueId()
    {
        var id = new byte[128];
        fixed (byte* p = id) PpGpu.Check(PpGpu.ppg_comm_unique_id(p));
        return id;
    }

    public void Dispose()
    {
        if (Comm != 0) PpGpu.ppg_comm_free(Comm);
        PpGpu.ppg_close(Ctx);
    }
}

public sealed class GpuBatchedFASTQ : IEnumerable<FastqRecord>, IDisposable
{
    public GpuBatchedFASTQ(string indexPath, string gzipPath, bool enableSsdOptimization, int device = 0)
    {
        PpGpu.Check(PpGpu.ppg_index_deserialize(indexPath, out _Ix));   // IndexIO.Deserialize
        _Path = gzipPath;
        _Threads = enableSsdOptimization ? 16 : 8;   // LazyFileReader: 8 FileStreams vs 1
        PpGpu.Check(PpGpu.ppg_open(device, out _Ctx));
        _OwnCtx = true;
    }

    /// <summary>This process is one rank of a multi-GPU job: Count() decodes the rank's share and
    /// gathers every rank's counts; enumeration yields this rank's share of the records (the chunk
    /// range ppg_partition gives it), so the ranks' records in rank order are the file's.</summary>
    public GpuBatchedFASTQ(string indexPath, string gzipPath, GpuJob job)
    {
        PpGpu.Check(PpGpu.ppg_index_deserialize(indexPath, out _Ix));
        _Path = gzipPath;
        _Threads = 16;
        _Ctx = job.Ctx;
        _Job = job;
    }

    private readonly nint _Ix, _Ctx;
    private readonly bool _OwnCtx;
    private readonly string _Path;
    private readonly int _Threads;
    private readonly GpuJob? _Job;

    /// <summary>Text per streamed batch.  ppg_cursor keeps up to five batches in flight, each slot
    /// ~1.13 x BatchBytes + its compressed bytes of pinned host memory (4 GiB: ~28 GB in all; the
    /// library drops slots where that exceeds half the available memory).  Any size: each chunk is
    /// copied into its own managed array (a chunk is below 2^31 bytes, ppg_index_validate), so a
    /// batch may exceed a managed array's limit.</summary>
    public long BatchBytes
    {
        get => _BatchBytes;
        set => _BatchBytes = value > 0 ? value : throw new ArgumentOutOfRangeException(nameof(value));
    }
    private long _BatchBytes = 4L << 30;

    /// <summary>Enumerable.Count over the records (Decompressor/Program.cs:48-52), without
    /// materialising them: one GPU streams the file, a multi-GPU job gathers every rank's counts.</summary>
    public unsafe long Count()
    {
        int chunks = PpGpu.ppg_index_count(_Ix) - 1;
        long total;
        if (_Job != null)
            PpGpu.Check(PpGpu.ppg_dist_decompress_all(_Ctx, _Job.Comm, _Ix, _Path, 0, null, null, out total));
        else
            PpGpu.Check(PpGpu.ppg_file_decompress_all(_Ctx, _Ix, _Path, 0, chunks, 0, _Threads, null, out total,
                                                      out _));
        return total;
    }

    // an iterator may not contain unsafe code: the batch is read by NextBatch, the records yielded here
    public IEnumerator<FastqRecord> GetEnumerator()
    {
        var (first, n) = ChunkRange();
        PpGpu.Check(PpGpu.ppg_cursor_open(_Ctx, _Ix, _Path, first, n, BatchBytes, _Threads, out var cur));
        try
        {
            while (true)
            {
                var recs = NextBatch(cur);
                if (recs == null) yield break;
                foreach (var r in recs) yield return r;
            }
        }
        finally
        {
            PpGpu.ppg_cursor_close(cur);
        }
    }

    // The chunks this enumerator streams: all of them, or (multi-GPU job) this rank's share
    private unsafe (int first, int n) ChunkRange()
    {
        int chunks = PpGpu.ppg_index_count(_Ix) - 1;
        if (_Job == null) return (0, chunks);
        var bounds = new int[_Job.NRanks + 1];
        fixed (int* b = bounds) PpGpu.Check(PpGpu.ppg_partition(_Ix, 0, chunks, _Job.NRanks, b));
        return (bounds[_Job.Rank], bounds[_Job.Rank + 1] - bounds[_Job.Rank]);
    }

    // The next batch's records, or null after the last batch.  Each chunk's raw bytes are copied
    // into a managed array of their own (the pinned batch is reused by a later ppg_cursor_next) that
    // its records slice; a chunk's raw_k is below 2^31 bytes (ppg_index_validate), a batch need not be.
    private static unsafe FastqRecord[]? NextBatch(nint cur)
    {
        int rc = PpGpu.ppg_cursor_next(cur, out var b);
        if (rc == (int)ZResult.STREAM_END) return null;
        PpGpu.Check(rc);
        var recs = new FastqRecord[b.NRecords];
        long o = 0;
        for (int k = 0; k < b.NChunks; k++)
        {
            var chunk = new byte[b.RawOff[k + 1] - b.RawOff[k]];
            new ReadOnlySpan<byte>(b.Text + b.RawOff[k], chunk.Length).CopyTo(chunk);
            var raw = new Memory<byte>(chunk);
            uint start = 0;   // Parsing.cs:19 -- the first record starts at raw[0] ('@' skipped)
            for (long j = b.RecOff[k]; j < b.RecOff[k + 1]; j++)
            {
                uint* d = b.Desc + 4 * j;
                // Parsing.cs:37-40: Identifier=[r+1,n1) Sequence=[n1+1,n2) Other=[n2+2,n3) Quality=[n3+1,n4)
                recs[o++] = new FastqRecord(null!,
                    raw.Slice((int)start + 1, (int)(d[0] - start - 1)),
                    raw.Slice((int)d[0] + 1, (int)(d[1] - d[0] - 1)),
                    raw.Slice((int)d[1] + 2, (int)(d[2] - d[1] - 2)),
                    raw.Slice((int)d[2] + 1, (int)(d[3] - d[2] - 1)));
                start = d[3] + 1;
            }
        }
        return recs;
    }

    IEnumerator IEnumerable.GetEnumerator() => GetEnumerator();

    public void Dispose()
    {
        PpGpu.ppg_index_free(_Ix);
        if (_OwnCtx) PpGpu.ppg_close(_Ctx);
    }
}

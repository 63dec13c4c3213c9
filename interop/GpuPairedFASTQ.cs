// interop/GpuPairedFASTQ.cs — paired-end reads over libppgpu (interop/PpGpu.cs): record-aligned pair
// chunks of two mate files (BASELINE configs[4]; the reference names the goal only, README.md:9).
//
//  * both files are decoded on one GPU (ppg_shard_create + ppg_shard_run over each index's chunks)
//    and paired on the device by ppg_pairs_check: spot keys, the records the reference parses twice
//    dropped (SURVEY Q1), keys compared -- a file pair that is not a read pair throws before any pair
//    is handed out;
//  * pair chunk j = pairs [j*K, (j+1)*K): the library packs both halves on the device window by
//    window (ppg_pairs_emit_begin / _next: each half is its records' bytes back to back + one
//    descriptor per record, the layout of one chunk's raw text), and each half crosses to the host
//    in one copy (ppg_pairs_copy_chunk), whose FastqRecords are cut as Parsing.cs:23-47 cuts them;
//  * a multi-GPU job (GpuJob) checks its ranks' shards together (CheckDistributed): every key moves to
//    the rank owning its pair number over the library's RCCL communicator; EmitDistributed then hands
//    each rank the pair chunks that start in its R1 range, the mates' records moved to it over RCCL.
// (Source only: no .NET SDK in this image; tests/test_interop_cs.py checks the externs it uses.)
using System;
using System.Collections;
using System.IO;
using ParallelParsing.Common;
using ParallelParsing.Interop;

namespace ParallelParsing;

public sealed unsafe class GpuPairedFASTQ : IEnumerable<(FastqRecord R1, FastqRecord R2)>, IDisposable
{
    public GpuPairedFASTQ(string index1, string gz1, string index2, string gz2, int pairChunk = 50_000, int device = 0)
    {
        _K = pairChunk > 0 ? pairChunk : throw new ArgumentOutOfRangeException(nameof(pairChunk));
        PpGpu.Check(PpGpu.ppg_open(device, out _Ctx));
        _Files = new[] { Open(index1, gz1), Open(index2, gz2) };
        PpGpu.Check(PpGpu.ppg_pairs_create(out _Pairs));
        PpGpu.Check(PpGpu.ppg_pairs_check(_Pairs, _Files[0].Shard, _Files[1].Shard, 0, out _Result));
        if (_Result.Records[0] != _Result.Records[1] || _Result.Mismatches != 0)
            throw new InvalidDataException(
                $"not a read pair: {_Result.Records[0]} vs {_Result.Records[1]} records, {_Result.Mismatches} " +
                $"mismatched pairs, first at pair {_Result.FirstBad} (spots {_Result.FirstKeys[0]} vs {_Result.FirstKeys[1]})");
    }

    /// <summary>ppg_pairs_check for the shards of one rank of a multi-GPU job (rank r holds R1 and R2
    /// shards of its own ppg_partition ranges): every rank gets the same result.</summary>
    public static PpgPairResult CheckDistributed(GpuJob job, nint shardR1, nint shardR2)
    {
        PpGpu.Check(PpGpu.ppg_pairs_create(out var p));
        try
        {
            PpGpu.Check(PpGpu.ppg_pairs_check(p, shardR1, shardR2, job.Comm, out var r));
            return r;
        }
        finally
        {
            PpGpu.ppg_pairs_free(p);
        }
    }

    private sealed class File1
    {
        public nint Index, Shard;
        public long[] Bases = Array.Empty<long>();   // record base of every chunk (ppg_shard_record_base)
    }

    private readonly nint _Ctx, _Pairs;
    private readonly File1[] _Files;
    private readonly PpgPairResult _Result;
    private readonly int _K;

    public long Count() => _Result.Pairs;
    public long Chunks => (_Result.Pairs + _K - 1) / _K;

    private File1 Open(string indexPath, string gzPath)
    {
        var f = new File1();
        PpGpu.Check(PpGpu.ppg_index_deserialize(indexPath, out f.Index));   // IndexIO.Deserialize
        int n = PpGpu.ppg_index_count(f.Index) - 1;
        PpGpu.Check(PpGpu.ppg_index_point(f.Index, 0, out _, out long i0, out _, out _));
        PpGpu.Check(PpGpu.ppg_index_point(f.Index, n, out _, out long i1, out _, out _));
        // the compressed range LazyFileReader would read, [Index[0].Input-1, Index[n].Input-1]
        var comp = new byte[i1 - i0 + 1];
        using (var fs = File.OpenRead(gzPath))
        {
            fs.Position = i0 - 1;
            fs.ReadExactly(comp);
        }
        fixed (byte* c = comp)
            PpGpu.Check(PpGpu.ppg_shard_create(_Ctx, f.Index, 0, n, c, comp.LongLength, 0, 0, out f.Shard));
        PpGpu.Check(PpGpu.ppg_shard_run(f.Shard));
        f.Bases = new long[n];
        fixed (long* b = f.Bases) PpGpu.Check(PpGpu.ppg_shard_record_base(f.Shard, b));
        return f;
    }

    /// <summary>Every pair chunk in order: (j, R1 records, R2 records), pairs [j*K, min((j+1)*K, Count)),
    /// from the library's device-packed windows (ppg_pairs_emit_next).</summary>
    public IEnumerable<(long J, FastqRecord[] R1, FastqRecord[] R2)> PairChunks(long windowBytes = 0)
    {
        PpGpu.Check(PpGpu.ppg_pairs_emit_begin(_Pairs, _Files[0].Shard, _Files[1].Shard, 0, _K, windowBytes));
        for (;;)
        {
            int rc = PpGpu.ppg_pairs_emit_next(_Pairs, out long j0, out long j1);
            if (rc == 1) yield break;   // PPG_STREAM_END
            PpGpu.Check(rc);
            for (long j = j0; j < j1; j++) yield return (j, Half(_Pairs, j, 0), Half(_Pairs, j, 1));
        }
    }

    /// <summary>A multi-GPU job's pair chunks on this rank (after CheckDistributed on the same shards):
    /// the ones that start in its R1 range; every rank must call it (the first window is collective).</summary>
    public static IEnumerable<(long J, FastqRecord[] R1, FastqRecord[] R2)> EmitDistributed(GpuJob job, nint pairs,
        nint shardR1, nint shardR2, int pairChunk)
    {
        PpGpu.Check(PpGpu.ppg_pairs_emit_begin(pairs, shardR1, shardR2, job.Comm, pairChunk, 0));
        for (;;)
        {
            int rc = PpGpu.ppg_pairs_emit_next(pairs, out long j0, out long j1);
            if (rc == 1) yield break;
            PpGpu.Check(rc);
            for (long j = j0; j < j1; j++) yield return (j, Half(pairs, j, 0), Half(pairs, j, 1));
        }
    }

    /// <summary>Pair chunks of two shards that have not run (each with ppg_shard_set_keys), the windows
    /// driving their run (ppg_pairs_emit_run): every output batch decoded once and its halves packed
    /// while resident -- for shards larger than HBM -- then the check over the keys they wrote.</summary>
    public static IEnumerable<(long J, FastqRecord[] R1, FastqRecord[] R2)> EmitRun(nint pairs, nint shardR1,
        nint shardR2, int pairChunk, long windowBytes = 0)
    {
        PpGpu.Check(PpGpu.ppg_pairs_emit_run(pairs, shardR1, shardR2, pairChunk, windowBytes));
        for (;;)
        {
            int rc = PpGpu.ppg_pairs_emit_next(pairs, out long j0, out long j1);
            if (rc == 1) break;
            PpGpu.Check(rc);
            for (long j = j0; j < j1; j++) yield return (j, Half(pairs, j, 0), Half(pairs, j, 1));
        }
        PpGpu.Check(PpGpu.ppg_pairs_check(pairs, shardR1, shardR2, 0, out var r));
        if (r.Mismatches != 0) throw new InvalidDataException($"R1/R2 pairing broken at pair {r.FirstBad}");
    }

    // one half: its bytes and descriptors in one copy each, FastqRecords over them
    private static FastqRecord[] Half(nint pairs, long j, int file)
    {
        PpGpu.Check(PpGpu.ppg_pairs_chunk(pairs, j, file, out _, out long len, out _, out long n));
        var raw = new byte[len];
        var desc = new uint[4 * n];
        fixed (byte* b = raw)
        fixed (uint* d = desc)
            PpGpu.Check(PpGpu.ppg_pairs_copy_chunk(pairs, j, file, b, len, out _, d, n, out _));
        var outp = new FastqRecord[n];
        var m = new Memory<byte>(raw);
        uint start = 0;   // Parsing.cs:19: raw[start] is the '@'
        for (long i = 0; i < n; i++)
        {
            outp[i] = new FastqRecord(null!,
                m.Slice((int)start + 1, (int)(desc[4 * i] - start - 1)),
                m.Slice((int)desc[4 * i] + 1, (int)(desc[4 * i + 1] - desc[4 * i] - 1)),
                m.Slice((int)desc[4 * i + 1] + 2, (int)(desc[4 * i + 2] - desc[4 * i + 1] - 2)),
                m.Slice((int)desc[4 * i + 2] + 1, (int)(desc[4 * i + 3] - desc[4 * i + 2] - 1)));
            start = desc[4 * i + 3] + 1;
        }
        return outp;
    }

    public IEnumerator<(FastqRecord R1, FastqRecord R2)> GetEnumerator()
    {
        foreach (var (_, a, b) in PairChunks())
            for (int i = 0; i < a.Length; i++) yield return (a[i], b[i]);
    }

    IEnumerator IEnumerable.GetEnumerator() => GetEnumerator();

    public void Dispose()
    {
        PpGpu.ppg_pairs_free(_Pairs);
        foreach (var f in _Files)
        {
            PpGpu.ppg_shard_free(f.Shard);
            PpGpu.ppg_index_free(f.Index);
        }
        PpGpu.ppg_close(_Ctx);
    }
}

// interop/GpuPairedFASTQ.cs — paired-end reads over libppgpu (interop/PpGpu.cs): record-aligned pair
// chunks of two mate files (BASELINE configs[4]; the reference names the goal only, README.md:9).
//
//  * both files are decoded on one GPU (ppg_shard_create + ppg_shard_run over each index's chunks)
//    and paired on the device by ppg_pairs_check: spot keys, the records the reference parses twice
//    dropped (SURVEY Q1), keys compared -- a file pair that is not a read pair throws before any pair
//    is handed out;
//  * pair chunk j = pairs [j*K, (j+1)*K): ppg_pairs_records maps pair numbers to each shard's record
//    numbers, whose FastqRecords are cut from raw_k = offset_k ++ chunk_k as Parsing.cs:23-47 cuts them;
//  * a multi-GPU job (GpuJob) checks its ranks' shards together (CheckDistributed): every key moves to
//    the rank owning its pair number over the library's RCCL communicator.
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

    /// <summary>(R1 records, R2 records) of pair chunk j: pairs [j*K, min((j+1)*K, Count)).</summary>
    public (FastqRecord[] R1, FastqRecord[] R2) PairChunk(long j)
    {
        long lo = j * _K, hi = Math.Min(lo + _K, _Result.Pairs);
        if (j < 0 || lo >= hi) throw new ArgumentOutOfRangeException(nameof(j));
        return (Records(0, lo, hi), Records(1, lo, hi));
    }

    private FastqRecord[] Records(int file, long lo, long hi)
    {
        var f = _Files[file];
        var rec = new long[hi - lo];
        fixed (long* r = rec) PpGpu.Check(PpGpu.ppg_pairs_records(_Pairs, file, lo, hi, r));
        var outp = new FastqRecord[rec.Length];
        int cached = -1;
        byte[] raw = Array.Empty<byte>();
        uint[] desc = Array.Empty<uint>();
        for (long i = 0; i < rec.Length; i++)
        {
            int k = Array.BinarySearch(f.Bases, rec[i]);
            if (k < 0) k = ~k - 1;
            while (k + 1 < f.Bases.Length && f.Bases[k + 1] <= rec[i]) k++;   // chunks without records
            if (k != cached)
            {
                (raw, desc) = Chunk(f, k);
                cached = k;
            }
            long j = rec[i] - f.Bases[k];
            uint start = j == 0 ? 0u : desc[4 * j - 1] + 1;   // Parsing.cs:19: raw[start] is the '@'
            var m = new Memory<byte>(raw);
            outp[i] = new FastqRecord(null!,
                m.Slice((int)start + 1, (int)(desc[4 * j] - start - 1)),
                m.Slice((int)desc[4 * j] + 1, (int)(desc[4 * j + 1] - desc[4 * j] - 1)),
                m.Slice((int)desc[4 * j + 1] + 2, (int)(desc[4 * j + 2] - desc[4 * j + 1] - 2)),
                m.Slice((int)desc[4 * j + 2] + 1, (int)(desc[4 * j + 3] - desc[4 * j + 2] - 1)));
        }
        return outp;
    }

    // raw_k = offset_k ++ chunk_k and chunk k's descriptors
    private static (byte[] raw, uint[] desc) Chunk(File1 f, int k)
    {
        PpGpu.Check(PpGpu.ppg_index_point(f.Index, k, out long o0, out _, out _, out int olen));
        PpGpu.Check(PpGpu.ppg_index_point(f.Index, k + 1, out long o1, out _, out _, out _));
        var raw = new byte[olen + (o1 - o0)];
        new ReadOnlySpan<byte>(PpGpu.ppg_index_offset(f.Index, k), olen).CopyTo(raw);
        fixed (byte* p = raw)
            PpGpu.Check(PpGpu.ppg_shard_copy_chunk(f.Shard, k, p + olen, o1 - o0, out _));
        PpGpu.Check(PpGpu.ppg_shard_copy_records(f.Shard, k, null, 0, out long n));
        var desc = new uint[4 * n];
        fixed (uint* d = desc) PpGpu.Check(PpGpu.ppg_shard_copy_records(f.Shard, k, d, n, out _));
        return (raw, desc);
    }

    public IEnumerator<(FastqRecord R1, FastqRecord R2)> GetEnumerator()
    {
        for (long j = 0; j < Chunks; j++)
        {
            var (a, b) = PairChunk(j);
            for (int i = 0; i < a.Length; i++) yield return (a[i], b[i]);
        }
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

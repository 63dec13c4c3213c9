"""Per-chunk Decompress (ppg_decompress_chunk, README "Decompress") latency and throughput on a
synthetic member of the bench's shape (150 bp Generator reads, chunk = 10,000): T = 1 calls one
after another (PPG_CHUNK_VERBOSE=1 prints each launch's phases), then T threads, then the async
entry point when the library has it.  Run on the GPU box: python tools/chunk_latency.py [--records N]."""
import argparse
import ctypes as C
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parallelparsing_amd as pp   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2_600_000)
    ap.add_argument("--chunk", type=int, default=10_000)
    ap.add_argument("--threads", default="1,8,64")
    ap.add_argument("--repeat", type=int, default=2, help="throughput legs per setting (the first grows the buffers)")
    args = ap.parse_args()
    S = pp.synth()
    sz = S.ppg_synth_fastq_size(0, args.records, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(0, 0, args.records, 150, C.c_void_p(txt.ctypes.data), sz, 16)
    gzb = np.zeros(sz, np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 4 << 20, 16, C.c_void_p(gzb.ctypes.data), gzb.size)
    gz = gzb[:L].tobytes()
    ix = pp.Core.BuildDeflateIndex(gz, args.chunk)
    n = ix.Count - 1
    slices = []
    for k in range(n):
        _, i0, _, _ = ix.point_fields(k)
        _, i1, _, _ = ix.point_fields(k + 1)
        slices.append(np.frombuffer(gz[i0 - 1:i1], np.uint8))
    dev = pp.Device(0)
    print(f"{n} chunks of {args.chunk} records, {L / 1e6:.1f} MB gz", flush=True)
    for k in range(min(n, 3)):   # warm
        pp.Core.ExtractDeflateIndex(slices[k], ix, k, device=dev, with_records=True)
    ts = []
    for k in range(min(n, 12)):
        t = time.perf_counter()
        _, _, rec = pp.Core.ExtractDeflateIndex(slices[k], ix, k, device=dev, with_records=True)
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"T=1: ms per call {np.median(ts):.2f} (min {min(ts):.2f})", flush=True)
    for T in [int(x) for x in args.threads.split(",") if int(x) > 1 for _ in range(args.repeat)]:
        nxt, lock, cnt = [0], threading.Lock(), [0]
        m = min(n, 16 * T)

        def work():
            while True:
                with lock:
                    k = nxt[0]
                    nxt[0] += 1
                if k >= m:
                    return
                _, _, r = pp.Core.ExtractDeflateIndex(slices[k], ix, k, device=dev, with_records=True)
                with lock:
                    cnt[0] += len(r)
        before = dev.decompress_chunk_stats()
        th = [threading.Thread(target=work) for _ in range(T)]
        t = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        sec = time.perf_counter() - t
        after = dev.decompress_chunk_stats()
        print(f"T={T}: {cnt[0] / sec / 1e6:.2f} M records/s, {m} chunks in {sec * 1e3:.1f} ms, "
              f"{after['launches'] - before['launches']} launches", flush=True)
    if hasattr(pp.Core, "ExtractDeflateIndexAsync"):
        for depth in [d for d in (64, 256, 1024) for _ in range(args.repeat)]:
            m = min(n, depth)
            t = time.perf_counter()
            futs = [pp.Core.ExtractDeflateIndexAsync(slices[k], ix, k, device=dev) for k in range(m)]
            tot = sum(len(f.result()[2]) for f in futs)
            sec = time.perf_counter() - t
            print(f"async depth {m}: {tot / sec / 1e6:.2f} M records/s ({sec * 1e3:.1f} ms)", flush=True)


if __name__ == "__main__":
    main()

"""Where the ingest leg's time goes (one 8 GiB piece's read + copy took 299 ms
against ~175 ms for the others, in every run).  Builds the bench member, writes it to $TMPDIR as the
bench's ingest leg does, reports on which NUMA node the file's page-cache pages sit (one page per
64 MiB, faulted in through a read-only mapping and asked with move_pages(2), no migration) per piece,
then runs ppg_file_decompress_all twice with PPG_INGEST_VERBOSE=1 (pread vs pinned-slot waits per
piece on stderr) and the pinned -> device copy rate.

  python tools/ingest_probe.py [--seg-records N] [--repeats R] [--piece-gib G] [--variant v ...]
"""
import argparse
import ctypes as C
import json
import mmap
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SYS_move_pages = 279   # x86_64


def page_nodes(path, step=64 << 20):
    """(offset, node) for one page per `step` bytes of the file's page cache."""
    libc = C.CDLL(None, use_errno=True)
    libc.syscall.restype = C.c_long
    size = os.path.getsize(path)
    out = []
    with open(path, "rb") as f:
        m = mmap.mmap(f.fileno(), size, prot=mmap.PROT_READ)
        # the mapping's address (ctypes cannot take a read-only mmap's buffer): from /proc/self/maps
        m_addr = None
        with open("/proc/self/maps") as mp:
            for ln in mp:
                if path in ln:
                    a, b = (int(x, 16) for x in ln.split()[0].split("-"))
                    if b - a >= size - 4096:
                        m_addr = a
                        break
        if m_addr is None:
            return {"error": "mapping not found"}
        offs = list(range(0, size, step))
        for o in offs:
            m[o]   # fault the page in (a read-only mapping of the page-cache page)
        n = len(offs)
        pages = (C.c_void_p * n)(*[m_addr + o for o in offs])
        status = (C.c_int * n)()
        rc = libc.syscall(SYS_move_pages, 0, C.c_ulong(n), pages, None, status, 0)
        if rc != 0:
            return {"error": f"move_pages rc {rc} errno {C.get_errno()}"}
        out = list(zip(offs, list(status)))
        m.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seg-records", type=int, default=10_485_760)
    ap.add_argument("--repeats", type=int, default=51)
    ap.add_argument("--piece-gib", type=float, default=8.0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--variant", nargs="*", default=["plain:INDEX=plain", "noprio:INDEX=plain,COPY_PRIO=0"],
                    help="name:KEY=V,... -- INDEX=plain|tail, SLOTS, SLOT_MB, COPY_STREAMS (PPG_INGEST_*)")
    args = ap.parse_args()
    import parallelparsing_amd as pp
    from parallelparsing_amd.tiled import TiledFile
    t = time.time()
    tf = TiledFile(args.seg_records, args.repeats, 10000, threads=16)
    print(f"[probe] member built in {time.time() - t:.1f}s: {tf.file_len / 1e9:.2f} GB", file=sys.stderr, flush=True)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ppg_probe_{os.getpid()}.fastq.gz")
    res = {}
    try:
        t = time.perf_counter()
        with open(path, "wb") as f:
            for lo in range(0, tf.file_len, 1 << 30):
                f.write(tf.file_bytes(lo, min(tf.file_len, lo + (1 << 30))))
        res["write_s"] = time.perf_counter() - t
        nodes = page_nodes(path)
        if isinstance(nodes, dict):
            res["numa"] = nodes
        else:
            pb = int(args.piece_gib * (1 << 30))
            per = {}
            for o, nd in nodes:
                per.setdefault(o // pb, {}).setdefault(str(nd), 0)
                per[o // pb][str(nd)] += 1
            res["numa_pages_per_piece"] = per
            print(f"[probe] page-cache nodes per {args.piece_gib:g} GiB piece: {per}", file=sys.stderr, flush=True)
        pb = int(args.piece_gib * (1 << 30))
        plain = tf.index(0, tf.npoints)
        tail = tf.index(0, tf.npoints)   # side points for the last 2 pieces' chunks (bench.py's ingest leg)
        c0 = int(np.searchsorted(tf.p_input, tf.file_len - 2 * pb))
        tail.set_side_points(*tf.side_points(c0, tf.npoints, 8))
        dev = pp.Device(0)
        os.environ["PPG_INGEST_VERBOSE"] = "1"
        res["variants"] = {}
        for spec in args.variant:
            name, _, kv = spec.partition(":")
            env = dict(x.split("=") for x in kv.split(",") if x)
            ix = plain if env.pop("INDEX", "tail") == "plain" else tail
            for k in ("PPG_INGEST_SLOTS", "PPG_INGEST_SLOT_MB", "PPG_INGEST_COPY_STREAMS", "PPG_INGEST_COPY_PRIO"):
                os.environ.pop(k, None)
            os.environ.update({"PPG_INGEST_" + k: v for k, v in env.items()})
            dev.release_file_buffers()   # the staging shape is read when the buffers are made
            runs = []
            for _ in range(args.runs):
                print(f"[probe] variant {name}", file=sys.stderr, flush=True)
                _, tot, sec = pp.decompress_file(ix, path, device=dev, threads=args.threads, piece_bytes=pb)
                assert tot == tf.expected_records()
                runs.append(sec)
                print(f"[probe] {name}: {sec:.3f} s, {tot / sec / 1e6:.1f} M records/s", file=sys.stderr, flush=True)
            res["variants"][name] = runs
        dev.release_file_buffers()
        import torch
        n = 4 << 30
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        best = 0.0
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            d.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            best = max(best, n / (time.perf_counter() - t) / 1e9)
        res["pcie_h2d_GBps"] = best
        # the ingest's copy shapes: 128 / 512 MiB copies back to back from rotating pinned slots
        for mb in (128, 512):
            m = mb << 20
            best = 0.0
            for _ in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                for i in range(n // m):
                    d[i * m:(i + 1) * m].copy_(h[i * m:(i + 1) * m], non_blocking=True)
                torch.cuda.synchronize()
                best = max(best, n / (time.perf_counter() - t) / 1e9)
            res[f"pcie_h2d_GBps_{mb}MiB_copies"] = best
        # NUMA: the GPU's node, the pinned buffer's pages, the CPUs this process may run on
        try:
            nodes = {}
            for c in sorted(os.listdir("/sys/class/drm")):
                f = f"/sys/class/drm/{c}/device/numa_node"
                if c.startswith("card") and "-" not in c and os.path.exists(f):
                    nodes[c] = open(f).read().strip()
            res["drm_numa_nodes"] = nodes
            res["cpus_allowed"] = len(os.sched_getaffinity(0))
            libc = C.CDLL(None, use_errno=True)
            libc.syscall.restype = C.c_long
            step = 256 << 20
            offs = list(range(0, n, step))
            pages = (C.c_void_p * len(offs))(*[h.data_ptr() + o for o in offs])
            status = (C.c_int * len(offs))()
            rc = libc.syscall(SYS_move_pages, 0, C.c_ulong(len(offs)), pages, None, status, 0)
            res["pinned_page_nodes"] = list(status) if rc == 0 else f"rc {rc}"
        except OSError as e:
            res["numa_error"] = str(e)
    finally:
        if os.path.exists(path):
            os.remove(path)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""TEST INFRASTRUCTURE — generates tests/golden/ (committed small fixtures).

For every case: <name>.gz (input), <name>.json (the oracle's CreateIndex points: output/input/
bits, offset bytes, window SHA-256) and, for two small cases, <name>.gzi (IndexIO byte format);
<name>.json also holds (per-chunk decompressed length + SHA-256, per-chunk record count + SHA-256 of the
(n,4) uint32-LE record table from Parsing.Parse, whole-stream SHA-256, gzip trailer check).

The expected values come from the C oracle (oracle/oracle.c over zlib 1.2.11) and are
cross-checked here against two independent paths before being written:
  * Python's gzip module must decompress the file to the concatenation of the chunks;
  * oracle/oracle_py.py (a separate CreateIndex restatement) must produce identical points.

Run:  python oracle/make_golden.py   (writes tests/golden/)
"""
import ctypes as C
import gzip
import hashlib
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from oracle import oracle_py as OP  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
KEEP_GZI = ("one_record", "fixed_c100")


def synth_text(n, seed=1, read_len=150, first=0):
    from parallelparsing_amd._lib import synth
    S = synth()
    sz = S.ppg_synth_fastq_size(first, n, read_len)
    a = np.zeros(sz, np.uint8)
    assert S.ppg_synth_fastq(seed, first, n, read_len, C.c_void_p(a.ctypes.data), sz, 1) == sz
    return a.tobytes()


def gz_member(text, level=6, mem_level=8, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, 31, mem_level, strategy)
    return c.compress(text) + c.flush()


def pigz_member(text, piece):
    from parallelparsing_amd._lib import synth
    S = synth()
    t = np.frombuffer(text, np.uint8)
    out = np.zeros(len(text) + len(text) // 2 + 4096, np.uint8)
    n = S.ppg_synth_gzip(C.c_void_p(t.ctypes.data), t.size, 6, piece, 2, C.c_void_p(out.ctypes.data), out.size)
    assert n > 0
    return out[:n].tobytes()


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def cases():
    base = synth_text(2400, seed=11)
    small = synth_text(600, seed=12)
    yield "l6_c200", gz_member(base, 6), 200
    yield "l6_c20", gz_member(base, 6), 20
    yield "l1_c150", gz_member(base, 1), 150
    yield "l9_c300", gz_member(base, 9), 300
    yield "fixed_c100", gz_member(small, 6, strategy=zlib.Z_FIXED), 100
    yield "huffonly_c20", gz_member(small, 6, strategy=zlib.Z_HUFFMAN_ONLY), 20      # SURVEY Q1 duplicates
    yield "rle_c100", gz_member(small, 6, strategy=zlib.Z_RLE), 100
    yield "memlevel1_c10", gz_member(small, 6, mem_level=1), 10                     # tiny blocks, all bit offsets
    yield "stored_c50", gz_member(small, 0), 50                                     # stored blocks
    yield "pigz_c100", pigz_member(base, 131072), 100                               # sync-flush empty stored blocks
    yield "one_record", gz_member(synth_text(1, seed=3), 6), 10000
    yield "short_reads_c30", gz_member(synth_text(900, seed=5, read_len=36), 6), 30
    yield "long_reads_c10", gz_member(synth_text(120, seed=6, read_len=2000), 6), 10
    # CRLF line endings: '\r' stays inside fields (Parsing.cs:53-69, unlike SimpleDecompressor)
    yield "crlf_c100", gz_member(small.replace(b"\n", b"\r\n"), 6), 100
    # malformed: empty lines (R-P3 conditions fail -> serial state machine), '@' inside quality
    # strings, an empty '+' line, and a NUL byte (parse stops there)
    lines = small.split(b"\n")
    mal = []
    for i, ln in enumerate(lines):
        mal.append(ln)
        if i % 97 == 5:
            mal.append(b"")                              # empty line -> quirks of the skip rules
        if i % 53 == 7 and ln and ln[:1] in b"?!*":
            mal[-1] = ln[:20] + b"@" + ln[21:]          # Q2: '@' counted as a record by CreateIndex
    yield "malformed_c40", gz_member(b"\n".join(mal), 6, strategy=zlib.Z_HUFFMAN_ONLY), 40
    nul = bytearray(small)
    nul[len(nul) * 2 // 3] = 0
    yield "nul_c60", gz_member(bytes(nul), 6), 60
    emptyplus = small.replace(b"+SRR", b"+\nX", 3)
    yield "plusline_c50", gz_member(emptyplus, 6), 50


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    for name, gzb, chunk in cases():
        text = gzip.decompress(gzb)
        ix = O.build_index(gzb, chunk)
        cmb, pts_py = OP.build_index(gzb, chunk)
        pts = ix.points()
        assert [tuple(p) for p in pts_py] == pts and cmb == ix.chunk_max_bytes, name
        chunks = []
        cat = []
        for k in range(ix.count - 1):
            b = O.extract(gzb, ix, k)
            rec = O.parse(pts[k][4], b)
            cat.append(b)
            chunks.append({"out_len": len(b), "sha256": sha(b), "records": int(len(rec)),
                           "rec_sha256": sha(np.ascontiguousarray(rec, "<u4").tobytes()),
                           "first_record": [int(x) for x in rec[0]] if len(rec) else None})
        assert b"".join(cat) == text, name
        crc, isize = int.from_bytes(gzb[-8:-4], "little"), int.from_bytes(gzb[-4:], "little")
        assert crc == zlib.crc32(text) and isize == len(text) % (1 << 32), name
        with open(os.path.join(OUT, name + ".gz"), "wb") as f:
            f.write(gzb)
        if name in KEEP_GZI:   # IndexIO byte-format pins (windows make .gzi files large)
            ix.serialize(os.path.join(OUT, name + ".gzi"))
        meta = {"name": name, "chunksize": chunk, "gz_len": len(gzb), "text_len": len(text),
                "text_sha256": sha(text), "points": len(pts), "chunk_max_bytes": ix.chunk_max_bytes,
                "total_records": sum(c["records"] for c in chunks), "chunks": chunks,
                "bits": [p[2] for p in pts], "inputs": [p[1] for p in pts], "outputs": [p[0] for p in pts],
                "window_sha256": [sha(p[3]) for p in pts], "offsets_hex": [p[4].hex() for p in pts]}
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump(meta, f, indent=0)
        manifest.append(name)
        print(f"{name:18s} gz {len(gzb):8d} text {len(text):8d} points {len(pts):4d} "
              f"records {meta['total_records']:6d} bits {sorted(set(meta['bits']))}")
    # corrupted streams: flipped bytes inside chunk 1's compressed range.  "corrupt_err" is the
    # first flip position (scanning forward) where zlib reports an error; "corrupt_garbage" one
    # where it decodes to wrong bytes without error.  A conforming decoder must match both.
    gzb = gz_member(synth_text(600, seed=12), 6)
    ix = O.build_index(gzb, 100)
    _, i1, _, _, _ = ix.point(1)
    _, i2, _, _, _ = ix.point(2)
    found = {}
    for q in range(i1 + 8, i2 - 8, 37):
        bad = bytearray(gzb)
        for j in range(q, q + 6):
            bad[j] ^= 0x5A
        try:
            out = O.extract(bytes(bad), ix, 1)
            if "corrupt_garbage" not in found and out != O.extract(gzb, ix, 1):
                found["corrupt_garbage"] = (bytes(bad), 0, sha(out), len(out))
        except O.OracleError as e:
            if "corrupt_err" not in found:
                found["corrupt_err"] = (bytes(bad), e.code, None, None)
        if len(found) == 2:
            break
    corrupt = []
    with open(os.path.join(OUT, "corrupt_clean.gz"), "wb") as f:   # the index comes from this file
        f.write(gzb)
    for name, (bad, code, osha, olen) in sorted(found.items()):
        with open(os.path.join(OUT, name + ".gz"), "wb") as f:
            f.write(bad)
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump({"name": name, "chunksize": 100, "chunk": 1, "oracle_status": code,
                       "out_sha256": osha, "out_len": olen}, f)
        corrupt.append(name)
        print(name, "oracle status", code)
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump({"cases": manifest, "corrupt": corrupt,
                   "generator": "oracle/make_golden.py", "zlib": zlib.ZLIB_RUNTIME_VERSION}, f, indent=1)


if __name__ == "__main__":
    main()

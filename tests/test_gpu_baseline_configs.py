"""GPU parity at BASELINE.json's own sizes (no -m gpu test ran a BASELINE workload).

configs[1]: a 1 M-read synthetic .fastq.gz, chunk = 10,000 -- every chunk's bytes and record
            table against the oracle (Core.cs:133-192, Parsing.cs:11-51 restated over zlib 1.2.11),
            the whole output against the gzip trailer's CRC-32/ISIZE, one wave per chunk and split
            at every inner block start (bench.py --workload 1m), which must agree exactly.
configs[2]: the full ~50 GB member bench.py times (tiled: its text is known exactly), decoded in
            HBM as the bench does (one batch, tail split): every chunk's status, produced length and
            R-E5 end flags, the record count (with the reference's Q1 duplicates), and byte equality
            of all ~204 GB of output with the known text, compared on the device segment by segment.
"""
import ctypes as C
import os
import sys
import zlib

import numpy as np
import pytest

import parallelparsing_amd as pp
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _synth_gz(nrec, seed, threads=16):
    S = pp.synth()
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(seed, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, threads)
    gzb = np.zeros(sz // 2 + (1 << 20), np.uint8)
    L = S.ppg_synth_gzip(C.c_void_p(txt.ctypes.data), sz, 6, 4 << 20, threads, C.c_void_p(gzb.ctypes.data), gzb.size)
    assert L > 0
    return txt, gzb[:L].tobytes()


def test_configs1_one_million_reads_bit_exact(device):
    txt, gz = _synth_gz(1_000_000, 2024)
    assert len(gz) > 80e6                                    # ~93 MB of gzip, ~382 MB of text
    ix = pp.Core.BuildDeflateIndex(gz, 10000)
    oi = O.build_index(gz, 10000)
    assert ix.Count == oi.count and ix.Count > 90
    n = ix.Count - 1
    _, i0, _, _ = ix.point_fields(0)
    _, i1, _, _ = ix.point_fields(n)
    comp = np.frombuffer(gz[i0 - 1:i1], np.uint8)
    sh = pp.Shard(ix, comp, 0, n, device=device).run()
    r = sh.results()
    assert (r["status"] == 0).all()
    assert (r["flags"][:-1] & 7 == 0).all()                  # R-E5 on every non-last chunk
    crc, tot, pos = 0, 0, 0
    for k in range(n):
        b = sh.chunk_bytes(k)
        exp = O.extract(gz, oi, k)
        assert b.tobytes() == exp, k
        assert np.array_equal(sh.chunk_records(k), O.parse(oi.point(k)[4], exp)), k
        crc = zlib.crc32(b.tobytes(), crc)
        tot += int(r["records"][k])
        pos += len(b)
    assert crc == int.from_bytes(gz[-8:-4], "little") and pos % (1 << 32) == int.from_bytes(gz[-4:], "little")
    assert pos == txt.size
    exp_tot, exp_counts = O.decompress_all(gz, oi, threads=16)
    assert tot == sh.total_records == exp_tot
    assert (r["records"] == exp_counts).all()
    # split at every inner deflate block start (the GPU CreateIndex's side points): identical run
    gix = pp.Core.BuildDeflateIndexGpu(np.frombuffer(gz, np.uint8), 10000, device=device, side_bytes=1)
    assert gix.Count == ix.Count
    bits, outs, win = gix.side_points(0, n)
    assert bits.size > 5 * n
    sp = pp.Shard(ix, comp, 0, n, device=device).set_split(bits, outs, win).run()
    rs = sp.results()
    for key in r:
        assert (r[key] == rs[key]).all(), key
    whole = sp.copy_output(0, pos)
    assert np.array_equal(whole, txt)
    for k in range(0, n, 7):
        assert np.array_equal(sp.chunk_records(k), sh.chunk_records(k)), k


def test_configs2_full_50gb_member_on_device(device):
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from parallelparsing_amd.tiled import TiledFile
    tf = TiledFile(bench.SEG_RECORDS, bench.REPEATS, 10000, threads=16)   # bench.py's default workload
    assert tf.file_len > 49e9
    dev = torch.device("cuda", device.device)
    n = tf.npoints - 1
    lo, hi = int(tf.p_input[0]) - 1, int(tf.p_input[-1])
    comp = torch.empty(hi - lo + 256, dtype=torch.uint8, device=dev)
    comp[hi - lo:].zero_()
    tf.fill_device(comp, lo, hi)
    sh = pp.Shard(tf.index(0, tf.npoints), comp.data_ptr(), first=0, n=n, device=device, comp_on_device=True,
                  comp_len=hi - lo, out_capacity=192 << 30)
    assert sh.batches == 1
    args = type("A", (), {"split": 0, "tail_split": 8, "tail_gens": 0.5})()
    s, ksplit = bench.auto_split(args, bench.wave_slots(dev), n)
    if s > 1:
        sh.set_split(*tf.side_points(n - ksplit, n + 1, s))
    sh.run()
    del comp
    r = sh.results()
    assert (r["status"] == 0).all()
    assert (r["produced"] == np.diff(tf.p_output)).all()
    assert (r["flags"][:-1] & 7 == 0).all(), np.nonzero(r["flags"][:-1] & 7)[0][:10]
    assert sh.total_records == int(r["records"].sum()) == tf.expected_records()
    # all ~204 GB of output == the known text (one segment per compare, on the device)
    text = torch.from_numpy(tf.text).to(dev)
    tl = tf.text_len
    buf = torch.empty(tl, dtype=torch.uint8, device=dev)
    total = int(tf.p_output[-1] - tf.p_output[0])
    assert total == tl * tf.repeats
    for i in range(tf.repeats):
        sh.copy_output(i * tl, tl, buf)
        assert torch.equal(buf, text), f"segment {i} differs"

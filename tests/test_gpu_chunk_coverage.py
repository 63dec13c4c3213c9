"""Per-chunk Decompress (README "Decompress", ppg_decompress_chunk) on chunks of bench.py's own
50 GB workload whose block search once left them to the one-wave decode (r05):

- chunk 329: a false candidate whose range holds the real next block start, which is no candidate
  at all -- chained by a repair piece from that block end (a second, small pass 1);
- chunk 1023 as the LAST chunk of index(0, 1025): its end is known only as its slice's last byte
  (no R-E5 end check) and its last block ends inside that byte.

Each chunk's bytes must equal the tiled member's known text (the member is S^T, its text exact),
its record table the one-wave decode's (PPG_CHUNK_NO_FIND), and every chunk must have been split
by the search (ppg_decompress_chunk_split_stats), i.e. none fell back."""
import os
import sys

import numpy as np
import pytest

import parallelparsing_amd as pp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def seg():
    sys.path.insert(0, ROOT)
    import bench
    from parallelparsing_amd.tiled import TiledFile
    return TiledFile(bench.SEG_RECORDS, 1, 10000, threads=16)   # one segment of bench.py's member


def expected_bytes(tf, k):
    return tf.text[int(tf.p_output[k]) - int(tf.p_output[0]):int(tf.p_output[k + 1]) - int(tf.p_output[0])]


@pytest.mark.parametrize("ks", [list(range(324, 336)), list(range(1016, 1024))], ids=["repair", "index_end"])
def test_bench_chunks_all_split(seg, ks):
    tf = seg
    ix = tf.index(0, 1025)
    assert tf.p_bits[1024] != 0   # the index's last chunk ends inside a byte
    dev = pp.Device(0)
    before = dev.decompress_chunk_stats()
    got = {}
    for k in ks:
        sl = np.frombuffer(tf.file_bytes(int(tf.p_input[k]) - 1, int(tf.p_input[k + 1])), np.uint8)
        n, buf, rec = pp.Core.ExtractDeflateIndex(sl, ix, k, device=dev, with_records=True)
        exp = expected_bytes(tf, k)
        assert n == exp.size and np.array_equal(buf[:n], exp), k
        got[k] = (sl, rec)
    st = dev.decompress_chunk_stats()
    assert st["split_chunks"] - before["split_chunks"] == len(ks), (st, before)
    os.environ["PPG_CHUNK_NO_FIND"] = "1"
    try:
        for k in ks:
            sl, rec = got[k]
            _, _, rec1 = pp.Core.ExtractDeflateIndex(sl, ix, k, device=dev, with_records=True)
            assert np.array_equal(rec, rec1), k
    finally:
        os.environ.pop("PPG_CHUNK_NO_FIND", None)


def test_bench_chunks_one_launch(seg):
    """The same chunks queued together (one launch through the asynchronous entry point)."""
    tf = seg
    ix = tf.index(0, 1025)
    dev = pp.Device(0)
    ks = list(range(320, 340)) + list(range(1010, 1024))
    before = dev.decompress_chunk_stats()
    futs = [pp.Core.ExtractDeflateIndexAsync(
        np.frombuffer(tf.file_bytes(int(tf.p_input[k]) - 1, int(tf.p_input[k + 1])), np.uint8), ix, k, device=dev)
        for k in ks]
    for k, f in zip(ks, futs):
        n, buf, _ = f.result()
        exp = expected_bytes(tf, k)
        assert n == exp.size and np.array_equal(buf[:n], exp), k
    st = dev.decompress_chunk_stats()
    assert st["split_chunks"] - before["split_chunks"] == len(ks), (st, before)

"""Product host code (libppgpu.so, no GPU needed): CreateIndex and IndexIO against the golden
vectors and the reference's byte format (Common/IndexIO.cs)."""
import gzip
import hashlib
import os

import numpy as np
import pytest

import parallelparsing_amd as pp
from conftest import CASES, GOLDEN, load_case


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.mark.parametrize("name", CASES)
def test_create_index_matches_golden(name):
    meta, gz = load_case(name)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    assert ix.Count == meta["points"] and ix.ChunkMaxBytes == meta["chunk_max_bytes"]
    for i in range(ix.Count):
        p = ix[i]
        assert (p.Output, p.Input, p.Bits) == (meta["outputs"][i], meta["inputs"][i], meta["bits"][i])
        assert sha(p.Window) == meta["window_sha256"][i]
        assert p.offset.hex() == meta["offsets_hex"][i]


@pytest.mark.parametrize("name", ["one_record", "fixed_c100"])
def test_serialize_is_byte_identical_to_reference_format(name, tmp_path):
    meta, gz = load_case(name)
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    out = tmp_path / "x.gzi"
    pp.IndexIO.Serialize(ix, str(out))
    with open(os.path.join(GOLDEN, name + ".gzi"), "rb") as f:
        assert out.read_bytes() == f.read()


def test_build_from_file_and_roundtrip(tmp_path):
    meta, gz = load_case("memlevel1_c10")
    p = tmp_path / "x.gz"
    p.write_bytes(gz)
    ix = pp.Core.BuildDeflateIndex(str(p), meta["chunksize"])
    pp.IndexIO.Serialize(ix, str(tmp_path / "a.gzi"))
    back = pp.IndexIO.Deserialize(str(tmp_path / "a.gzi"))
    assert back.Count == ix.Count and back.ChunkMaxBytes == ix.ChunkMaxBytes
    for i in range(ix.Count):
        a, b = ix[i], back[i]
        assert (a.Output, a.Input, a.Bits, a.Window, a.offset) == (b.Output, b.Input, b.Bits, b.Window, b.offset)
    pp.IndexIO.Serialize(back, str(tmp_path / "b.gzi"))
    assert (tmp_path / "a.gzi").read_bytes() == (tmp_path / "b.gzi").read_bytes()


def test_from_points_roundtrip():
    import numpy as np
    meta, gz = load_case("rle_c100")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    pts = [ix[i] for i in range(ix.Count)]
    ix2 = pp.Index.from_points([p.Output for p in pts], [p.Input for p in pts], [p.Bits for p in pts],
                               np.frombuffer(b"".join(p.Window for p in pts), np.uint8),
                               [len(p.offset) for p in pts],
                               np.frombuffer(b"".join(p.offset for p in pts) or b"\0", np.uint8), ix.ChunkMaxBytes)
    for i in range(ix.Count):
        a, b = pts[i], ix2[i]
        assert (a.Output, a.Input, a.Bits, a.Window, a.offset) == (b.Output, b.Input, b.Bits, b.Window, b.offset)


def test_errors_mirror_zexception():
    meta, gz = load_case("l6_c200")
    with pytest.raises(pp.PpgError) as e:
        pp.Core.BuildDeflateIndex(gz[: len(gz) // 2], 200)   # truncated: Read returns 0 -> DATA_ERROR
    assert e.value.code == -3
    with pytest.raises(pp.PpgError) as e:
        pp.Core.BuildDeflateIndex(gzip.compress(b"A" * 70000, mtime=0), 10)
    assert e.value.code == -50
    with pytest.raises(pp.PpgError) as e:
        pp.IndexIO.Deserialize("/nonexistent/x.gzi")
    assert e.value.code == -51


def _index_with_deltas(outputs, inputs, bits=None, offset_len=None):
    n = len(outputs)
    bits = bits if bits is not None else [0] * n
    offset_len = offset_len if offset_len is not None else [0] * n
    offs = np.zeros(max(1, sum(offset_len)), np.uint8)
    return pp.Index.from_points(np.array(outputs, np.int64), np.array(inputs, np.int64), np.array(bits, np.int32),
                                np.zeros(n * 32768, np.uint8), np.array(offset_len, np.int32), offs[:sum(offset_len)])


def test_validate_rejects_chunks_too_large_for_the_kernels():
    """a chunk whose output reaches 2^31 bytes (the kernel's and the descriptors' 32-bit
    raw index; Core.cs:140 casts the same length to int) or whose compressed span reaches 2^32 bits
    is refused up front (PPG_UNSUPPORTED), before any device work -- never decoded short."""
    ok = _index_with_deltas([0, 1000, (1 << 31) - 40000], [10, 500, 900])
    ok.validate()
    big = _index_with_deltas([0, 1000, 1000 + (1 << 31)], [10, 500, 900])
    big.validate(0, 1)                                   # the first chunk alone is fine
    with pytest.raises(pp.PpgError) as e:
        big.validate()
    assert e.value.code == -53
    # the offset carry counts toward the raw index: 2^31 - 100 bytes + a 200-byte carry
    carry = _index_with_deltas([0, (1 << 31) - 100], [10, 500], offset_len=[200, 0])
    with pytest.raises(pp.PpgError) as e:
        carry.validate()
    assert e.value.code == -53
    span = _index_with_deltas([0, 1000], [10, 10 + (1 << 29)])   # 2^32 compressed bits
    with pytest.raises(pp.PpgError) as e:
        span.validate()
    assert e.value.code == -53
    bad = _index_with_deltas([0, 1000], [500, 10])                # Inputs out of order
    with pytest.raises(pp.PpgError) as e:
        bad.validate()
    assert e.value.code == -52


def test_host_create_index_rejects_bad_trailer_crc():
    """zlib's gzip mode (Core.cs:30, inflateInit2(47)) checks the trailer CRC-32: Z_DATA_ERROR."""
    meta, gz = load_case("l6_c20")
    crc = int.from_bytes(gz[-8:-4], "little") ^ 0x10
    bad = gz[:-8] + crc.to_bytes(4, "little") + gz[-4:]
    with pytest.raises(pp.PpgError) as e:
        pp.Core.BuildDeflateIndex(bad, meta["chunksize"])
    assert e.value.code == -3


def test_set_side_points_rejects_points_outside_their_chunk():
    """ppg_index_set_side_points checks every side point against the Points: strictly inside one
    chunk in output AND in compressed bits (a point outside its chunk's bit range made
    a shared Decompress launch fail every request in it).  Valid points are accepted."""
    meta, gz = load_case("l6_c200")
    ix = pp.Core.BuildDeflateIndex(gz, meta["chunksize"])
    assert ix.Count >= 3
    o0, i0, b0, _ = ix.point_fields(0)
    o1, i1, b1, _ = ix.point_fields(1)
    o2, i2, b2, _ = ix.point_fields(2)
    bit0, bit1, bit2 = 8 * i0 - b0, 8 * i1 - b1, 8 * i2 - b2
    w = np.zeros(32768, np.uint8)
    good = ((bit0 + bit1) // 2, (o0 + o1) // 2)
    ix.set_side_points([good[0]], [good[1]], w)          # inside chunk 0 in both: accepted
    bad = [((bit1 + bit2) // 2, good[1]),                # output in chunk 0, bits in chunk 1
           (bit0, good[1]),                              # at chunk 0's own start bit
           (bit1, good[1]),                              # at the next Point's bit
           (good[0], o1),                                # output exactly at a Point
           (good[0], o0 - 1 if o0 > 0 else -1)]          # before the first Point
    for b, o in bad:
        with pytest.raises(pp.PpgError) as e:
            ix.set_side_points([b], [o], w)
        assert e.value.code == pp._lib.PPG_ARG_ERROR, (b, o)

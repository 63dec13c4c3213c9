"""The oracle pinned: both restatements (oracle/oracle.c, oracle/oracle_py.py) against the
committed golden vectors, the gzip trailer and Python's zlib (CPU only)."""
import gzip
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

from conftest import CASES, CORRUPT, GOLDEN, load_case
from oracle import oracle as O
from oracle import oracle_py as OP


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.mark.parametrize("name", CASES)
def test_oracle_index_matches_golden(name):
    meta, gz = load_case(name)
    ix = O.build_index(gz, meta["chunksize"])
    pts = ix.points()
    assert len(pts) == meta["points"]
    assert [p[0] for p in pts] == meta["outputs"]
    assert [p[1] for p in pts] == meta["inputs"]
    assert [p[2] for p in pts] == meta["bits"]
    assert [sha(p[3]) for p in pts] == meta["window_sha256"]
    assert [p[4].hex() for p in pts] == meta["offsets_hex"]
    assert ix.chunk_max_bytes == meta["chunk_max_bytes"]


@pytest.mark.parametrize("name", CASES)
def test_second_restatement_agrees(name):
    meta, gz = load_case(name)
    cmb, pts = OP.build_index(gz, meta["chunksize"])
    assert [p[0] for p in pts] == meta["outputs"] and [p[1] for p in pts] == meta["inputs"]
    assert [p[2] for p in pts] == meta["bits"] and [p[4].hex() for p in pts] == meta["offsets_hex"]
    assert [sha(p[3]) for p in pts] == meta["window_sha256"] and cmb == meta["chunk_max_bytes"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_chunks_and_records(name):
    meta, gz = load_case(name)
    ix = O.build_index(gz, meta["chunksize"])
    cat = []
    for k, c in enumerate(meta["chunks"]):
        b = O.extract(gz, ix, k)
        assert len(b) == c["out_len"] and sha(b) == c["sha256"]
        rec = O.parse(ix.point(k)[4], b)
        assert len(rec) == c["records"]
        assert sha(np.ascontiguousarray(rec, "<u4").tobytes()) == c["rec_sha256"]
        cat.append(b)
    text = b"".join(cat)
    # whole-stream pins independent of the restatement: Python's gzip and the trailer
    assert text == gzip.decompress(gz)
    assert sha(text) == meta["text_sha256"]
    assert int.from_bytes(gz[-8:-4], "little") == zlib.crc32(text)
    assert int.from_bytes(gz[-4:], "little") == len(text) & 0xFFFFFFFF


def test_parse_well_formed_matches_plain_fastq_reading():
    """For well-formed 4-line FASTQ the state machine equals an independent line grouping."""
    meta, gz = load_case("l6_c200")
    text = gzip.decompress(gz)
    lines = text.split(b"\n")[:-1]
    rec = O.parse(b"", text)
    assert len(rec) == len(lines) // 4
    pos = 0
    for j in range(len(rec)):
        hdr, seq, plus, qual = lines[4 * j:4 * j + 4]
        n1, n2, n3, n4 = (int(x) for x in rec[j])
        assert text[pos + 1:n1] == hdr[1:] and text[n1 + 1:n2] == seq
        assert text[n2 + 2:n3] == plus[1:] and text[n3 + 1:n4] == qual
        pos = n4 + 1


def test_quirk_q1_duplicate_records():
    """a Point exactly at a record start re-emits that record in the next chunk."""
    meta, _ = load_case("stored_c50")
    assert meta["total_records"] == 601   # 600 distinct records, one duplicated at a boundary


def test_decompress_all_threads_agree():
    meta, gz = load_case("memlevel1_c10")
    ix = O.build_index(gz, meta["chunksize"])
    t1, c1 = O.decompress_all(gz, ix, threads=1)
    t4, c4 = O.decompress_all(gz, ix, threads=4, mode=1)
    assert t1 == t4 == meta["total_records"]
    assert list(c1) == list(c4) == [c["records"] for c in meta["chunks"]]


@pytest.mark.parametrize("name", CORRUPT)
def test_corrupt_fixture(name):
    meta, gz = load_case(name)
    with open(os.path.join(GOLDEN, "corrupt_clean.gz"), "rb") as f:
        ix = O.build_index(f.read(), meta["chunksize"])
    if meta["oracle_status"]:
        with pytest.raises(O.OracleError) as e:
            O.extract(gz, ix, meta["chunk"])
        assert e.value.code == meta["oracle_status"]
    else:
        b = O.extract(gz, ix, meta["chunk"])
        assert sha(b) == meta["out_sha256"]


def test_q4_offset_overflow():
    """more than 32 KiB without '@' -> IndexOutOfRangeException in CreateIndex."""
    gz = gzip.compress(b"A" * 70000, mtime=0)
    with pytest.raises(O.OracleError) as e:
        O.build_index(gz, 10)
    assert e.value.code == -50

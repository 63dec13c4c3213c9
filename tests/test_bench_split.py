"""bench.py's choice of split chunks (ppg_shard_set_split), host logic only: MI355X = 256 CUs x 32
resident waves.  Measured basis: DESIGN.md §5 and §7."""
import argparse

import pytest

import bench

SLOTS = 256 * 32


def args(split=0, tail_split=8, tail_gens="auto", split_gens=1):
    return argparse.Namespace(split=split, tail_split=tail_split, tail_gens=tail_gens, split_gens=split_gens)


@pytest.mark.parametrize("chunks,expect", [
    (52735, (8, 4096)),      # the default 50 GB step: only the last half-generation, into <= 8
    (26498, (8, 4096)),      # strong-scaling rank share at N = 2: the tail too (r02: 412.9 vs 435.8 ms split-all)
    (13249, (8, 8192)),      # N = 4, 1.6 generations: a whole generation (r04: 175.6 vs 188.9 ms for half)
    (20480, (8, 4096)),      # 2.5 generations: the half-generation tail again
    (6755, (8, 6755)),       # N = 8: under one generation, every chunk
    (2000, (25, 2000)),      # ~6 generations' worth of waves
    (97, (64, 97)),          # the 1 M-read file: every inner block start
    (1, (64, 1)),
])
def test_auto_split(chunks, expect):
    assert bench.auto_split(args(), SLOTS, chunks) == expect


def test_explicit_split_covers_every_chunk():
    assert bench.auto_split(args(split=3), SLOTS, 52735) == (3, 52735)
    assert bench.auto_split(args(split=1), SLOTS, 97) == (1, 97)


def test_tail_knobs():
    assert bench.auto_split(args(tail_split=1), SLOTS, 60000) == (1, 4096)   # off: S = 1
    assert bench.auto_split(args(tail_gens=2.0), SLOTS, 60000) == (8, 16384)
    assert bench.auto_split(args(tail_gens="0.5"), SLOTS, 13249) == (8, 4096)   # the r03 rule at N = 4
    assert bench.auto_split(args(split_gens=6), SLOTS, 26498) == (8, 26498)   # the r01 rule, floor 8


def test_tail2_split():
    a = args()
    a.tail2 = "64:0.25"                                         # the default since r04 (16 before)
    a.split = 8
    assert bench.tail2_split(a, SLOTS, 4096) == (64, 2048)     # N = 1: the last quarter generation into 64
    assert bench.tail2_split(a, SLOTS, 1000) == (64, 1000)     # fewer split chunks than that: all of them
    a.tail2 = "off"
    assert bench.tail2_split(a, SLOTS, 4096) == (8, 0)
    a.tail2, a.split = "4:0.25", 8                              # not finer than the split: no second stage
    assert bench.tail2_split(a, SLOTS, 4096) == (8, 0)

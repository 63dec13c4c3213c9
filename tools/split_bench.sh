#!/bin/bash
# Chunk splitting (ppg_shard_set_split) on one GPU: per-rank shares of strong scaling (--repeats
# 203/N) and the paired configuration, with and without side points.  Output: gpurun_out/sp_<tag>.json
set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sp_$tag.json 2> gpurun_out/sp_$tag.log || exit $?; python -c "import json; d=json.load(open('gpurun_out/sp_$tag.json')); print('$tag', round(d['value']/1e6,1), d['unit'], round(d['ms_per_step'],1), 'ms', d.get('kernel_ms_per_step'))"; }
# SPLIT_RUNS: space-separated tag:args items, '_' standing for a space inside args
for spec in ${SPLIT_RUNS:-share8:--repeats_26 share8s8:--repeats_26_--split_8}; do
  a=${spec#*:}
  run "${spec%%:*}" ${a//_/ }
done

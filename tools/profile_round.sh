#!/bin/bash
# Round profile of the bench workload (run on the GPU box through gpurun):
#   1. rocprofv3 --kernel-trace --stats over bench.py (2 steps)  -> gpurun_out/prof_stats/
#   2. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, one pass each (HBM traffic per launch)
# tools/traffic_summary.py turns the outputs into profiles/<tag>_* and profiles/traffic.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o prof --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/prof_stats.json 2> gpurun_out/prof_stats.log || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/prof_$c -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.log || exit $?
done

#!/bin/bash
# GPU CreateIndex at a 16 GiB pass-2 buffer: repeat the best piece size of tools/ix_sweep.sh and its neighbours
set -o pipefail
mkdir -p gpurun_out/ixs2
for pk in 512 640 512 768; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --create-index --ix-capacity-gib 16 --ix-piece-kib $pk > gpurun_out/ixs2/ix16_p${pk}_$RANDOM.json 2>> gpurun_out/ixs2/ix16.log || exit $?
done

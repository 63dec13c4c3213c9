#!/bin/bash
# r03 v5 round-end batch: GPU CreateIndex piece-size sweep at a 16 GiB pass-2 buffer (VERDICT r02
# next #7: <= 2.0 s with <= 16 GiB of scratch), then the full GPU suite and smoke() on this build.
set -o pipefail
mkdir -p gpurun_out/ixs
for pk in 0 512 384 256; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --create-index --ix-capacity-gib 16 --ix-piece-kib $pk > gpurun_out/ixs/ix16_p$pk.json 2> gpurun_out/ixs/ix16_p$pk.log || exit $?
done
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --create-index --ix-piece-kib 384 > gpurun_out/ixs/ixdef_p384.json 2> gpurun_out/ixs/ixdef_p384.log || exit $?
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03v5_gputest.txt 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v5_smoke.txt 2>&1

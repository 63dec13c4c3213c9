#!/bin/bash
# Round-4 scaling evidence on the one-GPU box:
#   1. bench.py --gpus 8 as a one-GPU rehearsal (8 ranks on cuda:0, gloo + the library's host
#      transport for the count gather): partition, auto/tail split, gather_pairs, count gather,
#      max-over-ranks timing and the line at world 8;
#   2. the N = 1 step and rank 0's share of the N = 2/4/8 strong split of the default member on
#      the shipped kernel (--share), plus tail-split variants at N = 8 (SHARE8_VARIANTS).
# Outputs gpurun_out/r04_<tag>.json (+ .log).  Stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out
summ() { python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r04_$1.json') if l.startswith('{')][-1]); print('$1', d['n_gpus'], round(d['value']/1e6,1), 'Mrec/s', round(d['ms_per_step'],2), 'ms', {k: round(v,2) for k,v in d['kernel_ms_per_step'].items()}, d['config'].get('waves_per_chunk'))"; }
if [ -z "$SKIP_W8" ]; then
  PPG_BENCH_ONE_DEVICE=1 PPG_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 8 --seg-records 40000 \
    --repeats 16 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest > gpurun_out/r04_w8.json 2> gpurun_out/r04_w8.log || exit $?
  summ w8
fi
run() {
  tag=$1; shift
  timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-ingest "$@" \
    > gpurun_out/r04_$tag.json 2> gpurun_out/r04_$tag.log || exit $?
  summ $tag
}
[ -z "$SKIP_N1" ] && run n1
for n in ${SHARES-2 4 8}; do run share$n --share $n; done
for spec in ${SHARE8_VARIANTS}; do
  a=${spec#*:}
  run "s8_${spec%%:*}" --share 8 ${a//_/ }
done
# VARIANTS: tag:args items for any share ('_' stands for a space inside args)
for spec in ${VARIANTS}; do
  a=${spec#*:}
  run "v_${spec%%:*}" ${a//_/ }
done
exit 0

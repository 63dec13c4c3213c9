set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04s2
# the block finder's prefilter with BFINAL = 0 (ppg_index.hip; the inflate object is unchanged):
# next_piece redoes the last piece from E when none starts past it; the GPU suite, then the per-chunk Decompress and CreateIndex legs
timeout -k 10 700 python -u -m pytest tests/test_index_gpu.py tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04s2/gputest.txt 2>&1
rc=$?; tail -2 gpurun_out/r04s2/gputest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04s2/gputest.txt | head -20; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04s2/smoke.txt 2>&1 || { tail -5 gpurun_out/r04s2/smoke.txt; exit 1; }
timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-enumerate --create-index > gpurun_out/r04s2/bench_chunk_ci.json 2> gpurun_out/r04s2/bench_chunk_ci.log || exit $?
python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r04s2/bench_chunk_ci.json') if l.startswith('{')][-1]
print(d['value']/1e6, d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])
print({k: (round(v['records_per_s']/1e6,2), round(v['ms_per_call'],2)) for k,v in d['decompress_chunk'].items() if isinstance(v,dict) and 'records_per_s' in v})
c=d['create_index']; print(c['seconds'], c.get('first_run_s'), c['phases_ms'])"

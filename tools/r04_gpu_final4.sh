set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f3
# r04 final build (pipelined loop for every round but the last 322 bytes, DecompressAll + CreateIndex pass 1):
# parity first, then the round profiles (summarised on the box), the default line and the
# 50 GB CreateIndex
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04f3/gputest.txt 2>&1
rc=$?; tail -2 gpurun_out/r04f3/gputest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04f3/gputest.txt | head -20; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f3/smoke.txt 2>&1 || { tail -5 gpurun_out/r04f3/smoke.txt; exit 1; }
tail -1 gpurun_out/r04f3/smoke.txt
bash tools/profile_round.sh || exit $?
bash tools/pmc_stalls.sh || exit $?
python3 tools/traffic_summary.py r04f3 > gpurun_out/r04f3/traffic_summary.txt 2>&1 || exit $?
python3 tools/stall_summary.py r04f3 > gpurun_out/r04f3/stall_summary.txt 2>&1 || exit $?
cp profiles/r04f3_* profiles/traffic.json profiles/inflate_stalls.json gpurun_out/r04f3/
rm -rf gpurun_out/prof_stats gpurun_out/prof_FETCH_SIZE gpurun_out/prof_WRITE_SIZE gpurun_out/stall_?
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04f3/bench_default.json 2> gpurun_out/r04f3/bench_default.log || exit $?
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04f3/bench_default.json') if l.startswith('{')][-1]; print(d['value']/1e6, d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['issue'] and d['roofline']['issue']['salu_per_cu_cycle'])"
timeout -k 10 300 python3 -u bench.py --create-index --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/r04f3/create_index.json 2> gpurun_out/r04f3/create_index.log || exit $?
du -sh gpurun_out
SKIP_W8=1 STEPS=5 SHARES="2 4 8" bash tools/r04_shares.sh || exit $?
mkdir -p gpurun_out/r04f3/shares && mv gpurun_out/r04_n1.* gpurun_out/r04_share*.* gpurun_out/r04f3/shares/

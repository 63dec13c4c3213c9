set -o pipefail
mkdir -p gpurun_out/r04q
# CreateIndex pass 1 through the pipelined HOT loop (PPG_IXPIPE): its GPU CreateIndex tests on that
# build, then the 50 GB CreateIndex timed on both builds, alternating
PPG_LIB_PATH=abtmp/ixp/libppgpu.so timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -v --timeout 400 --timeout-method thread > gpurun_out/r04q/ixp_index_tests.txt 2>&1 || { rc=$?; tail -30 gpurun_out/r04q/ixp_index_tests.txt; exit $rc; }
tail -1 gpurun_out/r04q/ixp_index_tests.txt
for i in 1 2; do
  for t in cur ixp; do
    PPG_LIB_PATH=abtmp/$t/libppgpu.so timeout -k 10 300 python3 -u bench.py --create-index --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/r04q/ci_${t}_$i.json 2> gpurun_out/r04q/ci_${t}_$i.log || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04q/ci_${t}_$i.json') if l.startswith('{')][-1]; c=d['create_index']; print('$t', $i, round(c['seconds'],3), c['phases_ms'])"
  done
done

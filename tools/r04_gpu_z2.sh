set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04z2
# r04 final build: the GPU suite log, the paired and CreateIndex legs, the world-8 rehearsal
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z2/smoke.txt 2>&1 || { tail -5 gpurun_out/r04z2/smoke.txt; exit 1; }
timeout -k 10 300 python3 -u bench.py --paired --steps 3 --warmup 1 > gpurun_out/r04z2/paired.json 2> gpurun_out/r04z2/paired.log || exit $?
tail -c 400 gpurun_out/r04z2/paired.json
timeout -k 10 300 python3 -u bench.py --create-index --steps 2 --warmup 1 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/r04z2/create_index.json 2> gpurun_out/r04z2/create_index.log || exit $?
tail -c 400 gpurun_out/r04z2/create_index.json
PPG_BENCH_ONE_DEVICE=1 PPG_DIST_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 8 --seg-records 40000 \
    --repeats 16 --steps 2 --warmup 1 --no-cpu-baseline --no-ingest > gpurun_out/r04z2/w8.json 2> gpurun_out/r04z2/w8.log || exit $?
tail -c 300 gpurun_out/r04z2/w8.json
du -sh gpurun_out

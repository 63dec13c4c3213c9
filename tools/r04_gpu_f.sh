set -o pipefail
mkdir -p gpurun_out
# r04 v1: the round-control A/B winner as the shipped kernel, the found-side-points fix
timeout -k 10 240 python -u -m pytest tests/test_gpu_chunk_threads.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r04v1_gputest_chunk.txt 2>&1 || { rc=$?; tail -40 gpurun_out/r04v1_gputest_chunk.txt; exit $rc; }
grep -E "found\]|passed|failed" gpurun_out/r04v1_gputest_chunk.txt | tail -3
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04v1_gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/r04v1_gputest.txt
case $rc in 0|1) ;; *) echo "suite rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 3 --steps 3 new=abtmp/new/libppgpu.so walk2=abtmp/walk2/libppgpu.so w8=abtmp/hotlwta8/libppgpu.so base=abtmp/base/libppgpu.so > gpurun_out/r04v1_ab.json 2> gpurun_out/r04v1_ab.log || { rc=$?; tail -20 gpurun_out/r04v1_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04v1_ab.log | tail -12
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04v1_bench_default.json 2> gpurun_out/r04v1_bench_default.log || exit $?
tail -c 600 gpurun_out/r04v1_bench_default.json

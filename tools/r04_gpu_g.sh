set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_paths.py -v --timeout 280 --timeout-method thread > gpurun_out/r04v2_benchpaths.txt 2>&1 || { rc=$?; tail -40 gpurun_out/r04v2_benchpaths.txt; exit $rc; }
tail -2 gpurun_out/r04v2_benchpaths.txt
timeout -k 10 420 python3 -u tools/ab_multi.py --rounds 3 --steps 3 r4=abtmp/r4/libppgpu.so walk2=abtmp/walk2/libppgpu.so cw0=abtmp/cw0/libppgpu.so cw0w2=abtmp/cw0w2/libppgpu.so prio2=abtmp/prio2/libppgpu.so base=abtmp/base/libppgpu.so > gpurun_out/r04v2_ab.json 2> gpurun_out/r04v2_ab.log || { rc=$?; tail -20 gpurun_out/r04v2_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04v2_ab.log | tail -18

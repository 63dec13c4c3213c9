set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 3 --steps 3 pipe=abtmp/pipe/libppgpu.so pbp=abtmp/pbp/libppgpu.so > gpurun_out/r04l_ab.json 2> gpurun_out/r04l_ab.log || { rc=$?; tail -20 gpurun_out/r04l_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04l_ab.log | tail -8

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 3 --steps 3 pbp3=abtmp/pbp3/libppgpu.so pbp3u=abtmp/pbp3u/libppgpu.so p3u=abtmp/p3u/libppgpu.so pipe=abtmp/pipe/libppgpu.so > gpurun_out/r04n_ab.json 2> gpurun_out/r04n_ab.log || { rc=$?; tail -20 gpurun_out/r04n_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04n_ab.log | tail -12

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab_multi.py --rounds 3 --steps 3 pipe=abtmp/pipe/libppgpu.so pbp=abtmp/pbp/libppgpu.so pbp3=abtmp/pbp3/libppgpu.so p2=abtmp/p2/libppgpu.so p2b=abtmp/p2b/libppgpu.so p3=abtmp/p3/libppgpu.so > gpurun_out/r04m_ab.json 2> gpurun_out/r04m_ab.log || { rc=$?; tail -20 gpurun_out/r04m_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04m_ab.log | tail -18

set -o pipefail
mkdir -p gpurun_out/r04o
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 3 --steps 3 fin=abtmp/fin/libppgpu.so lean=abtmp/lean/libppgpu.so leanu=abtmp/leanu/libppgpu.so leanup=abtmp/leanup/libppgpu.so finu=abtmp/finu/libppgpu.so > gpurun_out/r04o/ab.json 2> gpurun_out/r04o/ab.log || { rc=$?; tail -20 gpurun_out/r04o/ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04o/ab.log | tail -15
SKIP_W8=1 STEPS=5 SHARES="4 8" VARIANTS="s4t2:--share_4_--tail2_64:0.5 s4g1:--share_4_--tail-gens_1 s8sp16:--share_8_--split_16 s8t2:--share_8_--tail2_64:0.5" bash tools/r04_shares.sh || exit $?
mkdir -p gpurun_out/r04o/shares && mv gpurun_out/r04_n1.* gpurun_out/r04_share*.* gpurun_out/r04_v_*.* gpurun_out/r04o/shares/

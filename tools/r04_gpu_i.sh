set -o pipefail
mkdir -p gpurun_out
# diagnostics on the r04 kernel: per-phase round stamps and per-chunk path counts
AB_STEPS=1 bash tools/ab_bench.sh stamps abtmp/stamps/libppgpu.so stats abtmp/stats/libppgpu.so base abtmp/r4f/libppgpu.so || exit $?
grep -h "PPG_STAMPS\|PPG_STATS" gpurun_out/ab_stamps.log gpurun_out/ab_stats.log | head -12

#!/bin/bash
# Build a variant of libppgpu.so for tools/ab_bench.sh: tools/ab_build.sh <tag> [EXTRA flags...]
# -> abtmp/<tag>/libppgpu.so (+ its ppg_inflate.lint: the inline-asm wait-state check must pass).
# The sources are the working tree's csrc, compiled with EXTRA (e.g. -DPPG_R4_LIM).
set -e
tag=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/abtmp/$tag
rm -rf "$d"; mkdir -p "$d/csrc" "$root/abtmp"
cp "$root"/parallelparsing_amd/csrc/* "$d/csrc/"
ln -sfn "$root/tools" "$root/abtmp/tools"   # the lint's ../../tools path from abtmp/<tag>/csrc
ln -sfn "$root/include" "$root/abtmp/include"
make -s -j8 -C "$d/csrc" OUT=.. EXTRA="$*" ../libppgpu.so ../ppg_inflate.lint >/dev/null
echo "$tag: $(strings "$d/libppgpu.so" | grep -m1 '^inflate-') EXTRA=[$*]"

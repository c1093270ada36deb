#!/bin/bash
# Build an A/B variant of libtog.so with extra hipcc flags into ab_libs/<name>/libtog.so
# usage: tools/ab_build.sh <name> "<extra flags>"
set -e
name=$1; flags=$2
src="$(cd "$(dirname "$0")/.." && pwd)/trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd/csrc"
out="$(cd "$(dirname "$0")/.." && pwd)/ab_libs/$name"   # (gitignored; travels to the GPU box)
mkdir -p "$out"
cd "$out"
for f in tog_runtime.cpp $(cd "$src" && ls k_*.hip); do
  x=""; [ "$f" = tog_runtime.cpp ] && x="-x hip"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $flags $x -c "$src/$f" -o "${f%.*}.o" &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o libtog.so *.o
echo "$out/libtog.so"

#!/bin/bash
# ab_quad.sh <name> "<flags>": libtog.so A/B variant that recompiles only the quadrotor kernels with extra
# hipcc flags and links them with the main build's other objects -> ab_libs/<name>/libtog.so
set -e
name=$1; flags=$2
root="$(cd "$(dirname "$0")/.." && pwd)"
src="$root/trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd/csrc"
out="$root/ab_libs/$name"
mkdir -p "$out"
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $flags -c "$src/k_quadrotor.hip" -o "$out/k_quadrotor.o"
objs=$(cd "$src" && ls *.o | grep -v '^k_quadrotor.o$' | sed "s|^|$src/|")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$out/libtog.so" $objs "$out/k_quadrotor.o"
echo "$out/libtog.so"

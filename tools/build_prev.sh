#!/usr/bin/env bash
# Build the committed (HEAD or $1) kernel as build/libptgpu_${2:-prev}.so for same-box A/B runs.
set -e
rev=${1:-HEAD}
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" cpu-path-tracing_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/cpu-path-tracing_amd/build"
name=${2:-prev}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -shared \
    -o "$root/cpu-path-tracing_amd/build/libptgpu_$name.so" "$tmp/cpu-path-tracing_amd/csrc/ptg_render.hip" \
    $(ls "$tmp"/cpu-path-tracing_amd/csrc/ptg_multi.cpp 2>/dev/null) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo "built build/libptgpu_$name.so from $rev"

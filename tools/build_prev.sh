#!/usr/bin/env bash
# Build the committed (HEAD or $1) kernel as build/libptgpu_prev.so for same-box A/B runs.
set -e
rev=${1:-HEAD}
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" cpu-path-tracing_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/cpu-path-tracing_amd/build"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -shared \
    -o "$root/cpu-path-tracing_amd/build/libptgpu_prev.so" "$tmp/cpu-path-tracing_amd/csrc/ptg_render.hip"
rm -rf "$tmp"
echo "built build/libptgpu_prev.so from $rev"

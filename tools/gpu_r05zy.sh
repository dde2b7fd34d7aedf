#!/usr/bin/env bash
# Round 5: the fast and the exact mode on one box (HEAD; the exact bench line
# read 182.5 ms against r05zo's 175.3 -- box or code?), and the r05zo-era
# source built as build/libptgpu_r05zo.so.
tag=${1:-r05zy}
bash tools/gpu_ab.sh ${tag} "main r05zo" 2 "--steps 3 --warmup 1;--exact-math --steps 3 --warmup 1"

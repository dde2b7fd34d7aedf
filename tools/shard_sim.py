#!/usr/bin/env python3
"""Single-GPU estimate of the tile-sharded multi-GPU step (bench.py --gpus N).

Renders each of the N row-band shards of the bench frame one after another
on ONE GPU and times each (HIP events on the launch stream).  Each rank of an
N-GPU run renders exactly one of these shards, so the N-GPU kernel time is
max_k T_k and the strong-scaling efficiency of the render part is
T_1 / (N * max_k T_k).  The gather (24.9 MB over xGMI) is not included.
Usage: python tools/shard_sim.py [--counts 1 2 4 8] [--steps 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-path-tracing_amd"))

import torch  # noqa: E402

import ptgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--scene", default="box")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--band-rows", type=int, default=ptgpu.DEFAULT_BAND_ROWS)
    ap.add_argument("--chunk", type=int, default=0)
    args = ap.parse_args()
    W, H, samps = args.width, args.height, args.spp // 4
    scn = ptgpu.make_scene(args.scene, W, H)
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    stream = torch.cuda.current_stream()
    res = {}
    with ptgpu.Context(scn, cam, device=0) as ctx:
        for n in args.counts:
            rows = ptgpu.shard_rows(H, args.band_rows, n)
            slab = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
            times = []
            for k in range(n):
                p = ptgpu.make_params(W, H, samps, 2, ptgpu.DEFAULT_SEED, args.band_rows, k, n, args.chunk)
                ctx.render_device(slab, p, None, stream)  # warm-up
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(args.steps)]
                for a, b in ev:
                    a.record(stream)
                    ctx.render_device(slab, p, None, stream)
                    b.record(stream)
                torch.cuda.synchronize()
                times.append(min(a.elapsed_time(b) for a, b in ev))
            res[n] = {"max_ms": max(times), "min_ms": min(times), "shard_ms": [round(t, 2) for t in times]}
            print(f"N={n}: shard ms {res[n]['shard_ms']}", file=sys.stderr, flush=True)
    t1 = res[min(res)]["max_ms"] * min(res)
    for n in res:
        res[n]["efficiency_vs_first"] = round(t1 / (n * res[n]["max_ms"]), 4)
    print(json.dumps({"workload": f"{args.scene} {W}x{H} {args.spp}spp", "band_rows": args.band_rows,
                      "chunk": args.chunk, "shards": res}))


if __name__ == "__main__":
    main()
